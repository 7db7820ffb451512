// xorec_hip_bm.hpp -- the MI355X XOR-EC plugin for the reference's benchmark,
// as a maintainer adds it to src/algorithms/ next to XorecBenchmarkGpuCmp
// (xorec_gpu_cmp_bm.hpp:1-23), implementing AbstractBenchmark
// (src/algorithms/abstract_bm.hpp:18-88).
//
// ONE source, two builds (integration/Makefile):
//   * against the reference's UNMODIFIED headers and its own abstract_bm.cpp /
//     utils.cpp where /root/reference is mounted (linked in a temporary
//     directory, never shipped);
//   * against this repository's restatement of those headers
//     (integration/iface/) into erasure-code-benchmark_amd/xec/libxec_plugin.so,
//     which bin/xec_bench, bin/xec_multi_leg and the GPU tests run.
//
// The codec is libxec_hip.so's C ABI (include/xec.h); HIP allocations and
// copies go through hip_buffers.hpp.
#ifndef XOREC_HIP_BM_HPP
#define XOREC_HIP_BM_HPP

#include "abstract_bm.hpp"
#include "xec.h"
#include "xec_plugin_options.hpp"

class XorecBenchmarkHip : public AbstractBenchmark {
public:
  // The reference's registration (runners.cpp:43-45 style): XecPluginOptions{}.
  explicit XorecBenchmarkHip(const BenchmarkConfig& config);
  XorecBenchmarkHip(const BenchmarkConfig& config, const XecPluginOptions& options);
  ~XorecBenchmarkHip() noexcept override;
  XorecBenchmarkHip(const XorecBenchmarkHip&) = delete;
  XorecBenchmarkHip& operator=(const XorecBenchmarkHip&) = delete;

  void setup() noexcept override;
  int encode() noexcept override;
  int decode() noexcept override;
  void simulate_data_loss() noexcept override;
  bool check_for_corruption() const noexcept override;

  // Diagnostics for the harness (no reference counterpart): the batch's
  // stripes, the last codec status (xec_status) and the data blocks the
  // current erasure draw lost.
  size_t stripes() const noexcept { return m_chunks; }
  int last_status() const noexcept { return m_last_status; }
  size_t lost_data_blocks() const noexcept;

protected:
  void m_write_data_buffer() noexcept override;

private:
  using DevBuf = std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>>;
  XecPluginOptions m_opt;
  uint64_t m_round = 0;  ///< setup() count: a fresh seeded round per iteration
  DevBuf m_gpu_block_bitmap;  ///< device bitmap: xec_decode scratch / xec_erase input
  DevBuf m_gpu_bad;           ///< device count of invalid blocks
  DevBuf m_host_stage;        ///< pinned copy of the data (host payload / host check)
  hipStream_t m_stream = nullptr;
  int m_last_status = 0;
};

#endif  // XOREC_HIP_BM_HPP
