// abstract_bm.cpp -- the interface's default bodies on host buffers
// (restating src/algorithms/abstract_bm.cpp:4-60).
#include "abstract_bm.hpp"

#include <tuple>

// abstract_bm.cpp:4-18
AbstractBenchmark::AbstractBenchmark(const BenchmarkConfig& config) noexcept
    : m_threads(config.num_cpu_threads),
      m_message_size(config.message_size),
      m_block_size(config.block_size),
      m_chunk_data_blocks(std::get<1>(config.ec_params)),
      m_chunk_parity_blocks(std::get<0>(config.ec_params) - std::get<1>(config.ec_params)),
      m_chunk_tot_blocks(std::get<0>(config.ec_params)),
      m_chunks(config.message_size / (config.block_size * std::get<1>(config.ec_params))),
      m_chunk_data_size(config.block_size * std::get<1>(config.ec_params)),
      m_chunk_parity_size(config.block_size * m_chunk_parity_blocks),
      m_chunk_lost_blocks(config.num_lost_blocks),
      m_data_buf(make_unique_aligned<uint8_t>(m_chunks * m_chunk_data_size)),
      m_parity_buf(make_unique_aligned<uint8_t>(m_chunks * m_chunk_parity_size)),
      m_block_bitmap(make_unique_aligned<uint8_t>(m_chunks * m_chunk_tot_blocks)) {}

// abstract_bm.cpp:20-39
void AbstractBenchmark::simulate_data_loss() noexcept {
  for (size_t c = 0; c < m_chunks; ++c) {
    uint8_t* bitmap = m_block_bitmap.get() + c * m_chunk_tot_blocks;
    select_lost_blocks(m_chunk_data_blocks, m_chunk_parity_blocks, m_chunk_lost_blocks, bitmap);
    for (size_t i = 0; i < m_chunk_tot_blocks; ++i) {
      if (bitmap[i]) continue;
      uint8_t* block = i < m_chunk_data_blocks
                           ? m_data_buf.get() + c * m_chunk_data_size + i * m_block_size
                           : m_parity_buf.get() + c * m_chunk_parity_size +
                                 (i - m_chunk_data_blocks) * m_block_size;
      std::memset(block, 0, m_block_size);
    }
  }
}

// abstract_bm.cpp:41-50
bool AbstractBenchmark::check_for_corruption() const noexcept {
  const size_t blocks = m_chunks * m_chunk_data_blocks;
  for (size_t b = 0; b < blocks; ++b)
    if (!validate_block(m_data_buf.get() + b * m_block_size, m_block_size)) return false;
  return true;
}

// abstract_bm.cpp:52-60
void AbstractBenchmark::m_write_data_buffer() noexcept {
  const size_t blocks = m_chunks * m_chunk_data_blocks;
  for (size_t b = 0; b < blocks; ++b)
    if (write_validation_pattern(m_data_buf.get() + b * m_block_size, m_block_size) != 0)
      throw_error("Failed to write random checking packet.");
}
