// abstract_bm.cpp -- default behaviour of the plugin interface, on host
// buffers (reference src/algorithms/abstract_bm.cpp:4-61).  Plain C++: no HIP.
#include "abstract_bm.hpp"

#include <cstdlib>
#include <cstring>

#include "ec_utils.hpp"

namespace xec {

namespace {

void free_host(uint8_t* p) { std::free(p); }

size_t stripes_of(const BenchmarkConfig& c) {
  const size_t k = data_blocks(c);
  return c.block_size && k ? c.message_size / (c.block_size * k) : 0;
}

}  // namespace

Buffer make_host_buffer(size_t bytes) noexcept {
  if (bytes == 0) return Buffer(nullptr, free_host);
  const size_t rounded = (bytes + 63) / 64 * 64;  // aligned_alloc wants a multiple
  return Buffer(static_cast<uint8_t*>(std::aligned_alloc(64, rounded)), free_host);
}

// abstract_bm.cpp:4-18
AbstractBenchmark::AbstractBenchmark(const BenchmarkConfig& config) noexcept
    : m_threads(config.num_cpu_threads),
      m_message_size(config.message_size),
      m_block_size(config.block_size),
      m_chunk_data_blocks(data_blocks(config)),
      m_chunk_parity_blocks(parity_blocks(config)),
      m_chunk_tot_blocks(m_chunk_data_blocks + m_chunk_parity_blocks),
      m_chunks(stripes_of(config)),
      m_chunk_data_size(m_block_size * m_chunk_data_blocks),
      m_chunk_parity_size(m_block_size * m_chunk_parity_blocks),
      m_chunk_lost_blocks(config.num_lost_blocks),
      m_seed(config.seed),
      m_data_buf(make_host_buffer(m_chunks * m_chunk_data_size)),
      m_parity_buf(make_host_buffer(m_chunks * m_chunk_parity_size)),
      m_block_bitmap(make_host_buffer(m_chunks * m_chunk_tot_blocks)) {}

// abstract_bm.cpp:20-39: per stripe, pick a recoverable erasure set (at most
// one lost block per parity class) and zero the lost data and parity blocks.
void AbstractBenchmark::simulate_data_loss() noexcept {
  for (size_t c = 0; c < m_chunks; ++c) {
    uint8_t* bitmap = m_block_bitmap.get() + c * m_chunk_tot_blocks;
    uint8_t* data = m_data_buf.get() + c * m_chunk_data_size;
    uint8_t* parity = m_parity_buf.get() + c * m_chunk_parity_size;
    select_lost_blocks(m_chunk_data_blocks, m_chunk_parity_blocks, m_chunk_lost_blocks, bitmap,
                       round_seed(c));
    for (size_t i = 0; i < m_chunk_tot_blocks; ++i) {
      if (bitmap[i]) continue;
      uint8_t* blk = i < m_chunk_data_blocks ? data + i * m_block_size
                                             : parity + (i - m_chunk_data_blocks) * m_block_size;
      std::memset(blk, 0, m_block_size);
    }
  }
}

// abstract_bm.cpp:41-50: every data block still carries a valid payload.
bool AbstractBenchmark::check_for_corruption() const noexcept {
  const size_t nblocks = m_chunks * m_chunk_data_blocks;
  for (size_t b = 0; b < nblocks; ++b)
    if (!validate_block(m_data_buf.get() + b * m_block_size, m_block_size)) return false;
  return true;
}

// abstract_bm.cpp:52-61: a fresh validation payload in every data block.
void AbstractBenchmark::m_write_data_buffer() noexcept {
  const size_t nblocks = m_chunks * m_chunk_data_blocks;
  for (size_t b = 0; b < nblocks; ++b)
    write_validation_block(m_data_buf.get() + b * m_block_size, m_block_size, round_seed(b));
}

}  // namespace xec
