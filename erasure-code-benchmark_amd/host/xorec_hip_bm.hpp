// xorec_hip_bm.hpp -- the XOR-EC plugin on MI355X, through the C ABI of
// libxec_hip.so (include/xec.h).
//
// Drop-in sibling of the reference's XorecBenchmarkGpuCmp
// (src/algorithms/xorec_gpu_cmp_bm.{hpp,cpp}): same five virtuals, same batch
// layout, same pinned host bitmap + device bitmap scratch, one codec call per
// batch followed by a stream synchronise.  Differences, each a fix:
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

 private:
  void write_data_buffer() noexcept;

  hipStream_t m_stream = nullptr;
  uint8_t* m_data = nullptr;        // device, S*k*bs
  uint8_t* m_parity = nullptr;      // device, S*m*bs
  uint8_t* m_d_bitmap = nullptr;    // device scratch, S*(k+m)
  uint8_t* m_d_erase = nullptr;     // device copy of the erasure bitmap
  uint8_t* m_h_bitmap = nullptr;    // pinned host, S*(k+m)
  uint8_t* m_h_stage = nullptr;     // pinned host staging (host_validation only)
  uint32_t* m_d_bad = nullptr;      // device counter of corrupted blocks
  bool m_host_validation;
  uint64_t m_seed;
  uint64_t m_round = 0;             // bumps per setup(): fresh payload per iteration
  int m_last_status = 0;
};

}  // namespace xec
