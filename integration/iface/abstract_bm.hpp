// abstract_bm.hpp -- this repository's restatement of the reference's codec
// plugin interface, src/algorithms/abstract_bm.hpp:18-88: the same class name,
// the same virtual set (setup / encode / decode pure; simulate_data_loss,
// check_for_corruption and m_write_data_buffer with host-buffer defaults) and
// the same protected members, so that one plugin source compiles against
// either header (integration/Makefile).  Bodies: abstract_bm.cpp here.
#ifndef ABSTRACT_BM_HPP
#define ABSTRACT_BM_HPP

#include <cstdint>
#include <cstring>
#include <memory>

#include "bm_config.hpp"
#include "utils.hpp"

class AbstractBenchmark {
 public:
  virtual ~AbstractBenchmark() noexcept = default;
  virtual void setup() noexcept = 0;
  // 0 on success
  virtual int encode() noexcept = 0;
  // 0 on success; the losses were injected by simulate_data_loss before
  virtual int decode() noexcept = 0;
  // per stripe, a recoverable erasure set (select_lost_blocks) zeroed in place
  virtual void simulate_data_loss() noexcept;
  // true iff every data block passes validate_block
  virtual bool check_for_corruption() const noexcept;

 protected:
  // geometry from the config (m_chunks = message_size / (block_size * k)),
  // 64-B aligned host buffers for data, parity and the block bitmap
  explicit AbstractBenchmark(const BenchmarkConfig& config) noexcept;
  // a validation payload in every data block
  virtual void m_write_data_buffer() noexcept;

  size_t m_threads;
  size_t m_message_size;
  size_t m_block_size;

  size_t m_chunk_data_blocks;
  size_t m_chunk_parity_blocks;
  size_t m_chunk_tot_blocks;

  size_t m_chunks;

  size_t m_chunk_data_size;
  size_t m_chunk_parity_size;

  size_t m_chunk_lost_blocks;

  std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>> m_data_buf;
  std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>> m_parity_buf;
  std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>> m_block_bitmap;
};

#endif  // ABSTRACT_BM_HPP
