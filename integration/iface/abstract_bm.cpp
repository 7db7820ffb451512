// abstract_bm.cpp -- the interface's default bodies, on host buffers.  The
// behaviour restates src/algorithms/abstract_bm.cpp:4-60: the constructor
// derives the stripe geometry from the config and allocates aligned host
// buffers; the defaults erase, validate and fill those buffers per block.
#include "abstract_bm.hpp"

#include <tuple>

namespace {

// block `i` of stripe `s`: data blocks first, then the parity blocks
uint8_t* block_at(uint8_t* data, uint8_t* parity, size_t s, size_t i, size_t k, size_t m,
                  size_t bs) {
  return i < k ? data + (s * k + i) * bs : parity + (s * m + (i - k)) * bs;
}

}  // namespace

// abstract_bm.cpp:4-18.  ec_params is (total, data); stripes = whole stripes
// the message fills.
AbstractBenchmark::AbstractBenchmark(const BenchmarkConfig& config) noexcept
    : m_data_buf(nullptr, mm_deleter<uint8_t>),
      m_parity_buf(nullptr, mm_deleter<uint8_t>),
      m_block_bitmap(nullptr, mm_deleter<uint8_t>) {
  const size_t total = std::get<0>(config.ec_params);
  const size_t data = std::get<1>(config.ec_params);
  m_threads = config.num_cpu_threads;
  m_message_size = config.message_size;
  m_block_size = config.block_size;
  m_chunk_data_blocks = data;
  m_chunk_parity_blocks = total - data;
  m_chunk_tot_blocks = total;
  m_chunk_data_size = data * config.block_size;
  m_chunk_parity_size = (total - data) * config.block_size;
  m_chunks = config.message_size / m_chunk_data_size;
  m_chunk_lost_blocks = config.num_lost_blocks;
  m_data_buf = make_unique_aligned<uint8_t>(m_chunks * m_chunk_data_size);
  m_parity_buf = make_unique_aligned<uint8_t>(m_chunks * m_chunk_parity_size);
  m_block_bitmap = make_unique_aligned<uint8_t>(m_chunks * m_chunk_tot_blocks);
}

// abstract_bm.cpp:20-39: draw each stripe's losses, then zero every lost
// block, data or parity.
void AbstractBenchmark::simulate_data_loss() noexcept {
  const size_t k = m_chunk_data_blocks, m = m_chunk_parity_blocks;
  for (size_t s = 0; s < m_chunks; ++s) {
    uint8_t* row = m_block_bitmap.get() + s * m_chunk_tot_blocks;
    select_lost_blocks(k, m, m_chunk_lost_blocks, row);
    for (size_t i = 0; i < k + m; ++i)
      if (row[i] == 0)
        std::memset(block_at(m_data_buf.get(), m_parity_buf.get(), s, i, k, m, m_block_size), 0,
                    m_block_size);
  }
}

// abstract_bm.cpp:41-50: the batch is intact iff every data block validates.
bool AbstractBenchmark::check_for_corruption() const noexcept {
  const uint8_t* p = m_data_buf.get();
  const uint8_t* end = p + m_chunks * m_chunk_data_size;
  for (; p < end; p += m_block_size)
    if (!validate_block(p, m_block_size)) return false;
  return true;
}

// abstract_bm.cpp:52-60: a fresh payload per data block.
void AbstractBenchmark::m_write_data_buffer() noexcept {
  uint8_t* p = m_data_buf.get();
  uint8_t* end = p + m_chunks * m_chunk_data_size;
  for (; p < end; p += m_block_size)
    if (write_validation_pattern(p, m_block_size) != 0)
      throw_error("Failed to write random checking packet.");
}
