// abstract_bm.hpp -- the codec plugin interface the HIP plugin implements.
//
// Same contract as the reference's AbstractBenchmark
// (src/algorithms/abstract_bm.hpp:18-88): setup / encode / decode return-0-on-
// success / simulate_data_loss / check_for_corruption, a protected constructor
// from the BenchmarkConfig, and the batch geometry members the reference's
// plugins use (m_chunks = stripes = message_size / (block_size * k),
// abstract_bm.cpp:4-18).  Buffer ownership is left to the concrete plugin
// because the HIP plugin's buffers live in HBM.
#pragma once

#include "bm_config.hpp"

namespace xec {

class AbstractBenchmark {
 public:
  virtual ~AbstractBenchmark() noexcept = default;
  virtual void setup() noexcept = 0;
  virtual int encode() noexcept = 0;
  virtual int decode() noexcept = 0;
  virtual void simulate_data_loss() noexcept = 0;
  virtual bool check_for_corruption() const noexcept = 0;

 protected:
  explicit AbstractBenchmark(const BenchmarkConfig& config) noexcept
      : m_threads(config.num_cpu_threads),
        m_message_size(config.message_size),
        m_block_size(config.block_size),
        m_chunk_data_blocks(data_blocks(config)),
        m_chunk_parity_blocks(parity_blocks(config)),
        m_chunk_tot_blocks(m_chunk_data_blocks + m_chunk_parity_blocks),
        m_chunks(m_block_size && m_chunk_data_blocks
                     ? m_message_size / (m_block_size * m_chunk_data_blocks)
                     : 0),
        m_chunk_data_size(m_block_size * m_chunk_data_blocks),
        m_chunk_parity_size(m_block_size * m_chunk_parity_blocks),
        m_chunk_lost_blocks(config.num_lost_blocks) {}

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
};

}  // namespace xec
