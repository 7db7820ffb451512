// xorec_hip_bm.hpp -- the XOR-EC plugin on MI355X, through the C ABI of
// libxec_hip.so (include/xec.h).
//
// Drop-in sibling of the reference's XorecBenchmarkGpuCmp
// (src/algorithms/xorec_gpu_cmp_bm.{hpp,cpp}): same five virtuals, same batch
// layout, the base class's m_data_buf / m_parity_buf replaced by HBM
// allocations and m_block_bitmap by pinned host memory (as
// xorec_gpu_cmp_bm.cpp:6-18 does), a device bitmap scratch, one codec call per
// batch followed by a stream synchronise.  It overrides the base class's
// defaults (simulate_data_loss, check_for_corruption, m_write_data_buffer)
// because they touch buffers that now live in HBM.  Differences, each a fix:
//   - simulate_data_loss zeroes lost blocks with ONE kernel and synchronises,
//     instead of per-block cudaMemset calls that drain into the decode timer
//     (xorec_gpu_cmp_bm.cpp:71-89);
//   - parity is not destroyed by decode, so check_for_corruption may also
//     re-verify parity (it checks data blocks, as the reference does);
//   - seeds are explicit (config.seed), so every run is reproducible;
//   - the validation payload is written and checked on the device by default
//     (config.host_validation = true restores the host + copy path).
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <vector>

#include "abstract_bm.hpp"

namespace xec {

class XorecBenchmarkHip : public AbstractBenchmark {
 public:
  explicit XorecBenchmarkHip(const BenchmarkConfig& config);
  ~XorecBenchmarkHip() noexcept override;
  XorecBenchmarkHip(const XorecBenchmarkHip&) = delete;
  XorecBenchmarkHip& operator=(const XorecBenchmarkHip&) = delete;

  void setup() noexcept override;
  int encode() noexcept override;
  int decode() noexcept override;
  void simulate_data_loss() noexcept override;
  bool check_for_corruption() const noexcept override;

  size_t stripes() const { return m_chunks; }
  // Last status returned by the codec (xec_status), for diagnostics.
  int last_status() const { return m_last_status; }

 protected:
  void m_write_data_buffer() noexcept override;

 private:
  // m_data_buf: device S*k*bs; m_parity_buf: device S*m*bs; m_block_bitmap:
  // pinned host S*(k+m) (base-class members, replaced in the constructor)
  hipStream_t m_stream = nullptr;
  Buffer m_d_bitmap;   // device scratch for xec_decode, S*(k+m)
  Buffer m_d_erase;    // device copy of the erasure bitmap for xec_erase
  Buffer m_h_stage;    // pinned host staging (host_validation only)
  Buffer m_d_bad;      // device counter of corrupted blocks (4 B)
  bool m_host_validation;
  int m_last_status = 0;
};

}  // namespace xec
