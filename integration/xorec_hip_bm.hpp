// xorec_hip_bm.hpp -- the MI355X XOR-EC plugin for the reference's benchmark,
// written against the reference's UNMODIFIED plugin interface
// (src/algorithms/abstract_bm.hpp:18-88) as a maintainer would add it to
// src/algorithms/ next to XorecBenchmarkGpuCmp (xorec_gpu_cmp_bm.hpp:1-23).
//
// The codec is libxec_hip.so's C ABI (include/xec.h); HIP allocations and
// copies go through hip_buffers.hpp.  tests/test_reference_integration.py
// compiles this file with the reference's own abstract_bm.cpp and utils.cpp
// and links it against libxec_hip.so.
#ifndef XOREC_HIP_BM_HPP
#define XOREC_HIP_BM_HPP

#include "abstract_bm.hpp"
#include "xec.h"

class XorecBenchmarkHip : public AbstractBenchmark {
public:
  explicit XorecBenchmarkHip(const BenchmarkConfig& config);
  ~XorecBenchmarkHip() noexcept override;
  void setup() noexcept override;
  int encode() noexcept override;
  int decode() noexcept override;
  void simulate_data_loss() noexcept override;
  bool check_for_corruption() const noexcept override;

protected:
  void m_write_data_buffer() noexcept override;

private:
  std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>> m_gpu_block_bitmap;  ///< device bitmap / decode scratch
  std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>> m_gpu_bad;           ///< device count of invalid blocks
  hipStream_t m_stream = nullptr;
};

#endif  // XOREC_HIP_BM_HPP
