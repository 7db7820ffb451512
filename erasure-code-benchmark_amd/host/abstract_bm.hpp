// abstract_bm.hpp -- the codec plugin interface the HIP plugin implements.
//
// Same contract as the reference's AbstractBenchmark
// (src/algorithms/abstract_bm.hpp:18-88, abstract_bm.cpp:4-61):
//   * setup / encode / decode are pure virtual (0 = success);
//   * simulate_data_loss and check_for_corruption are virtual WITH default
//     bodies that work on host buffers: per stripe, select a recoverable
//     erasure set and zero those blocks; validate every data block's embedded
//     checksum (abstract_bm.cpp:20-50);
//   * the protected m_write_data_buffer hook writes the validation payload
//     into every data block (abstract_bm.cpp:52-61);
//   * the protected constructor derives the batch geometry from the
//     BenchmarkConfig (m_chunks = message_size / (block_size * k),
//     abstract_bm.cpp:4-18) and allocates 64-B-aligned host buffers for data,
//     parity and the block bitmap, which a device plugin replaces with its own
//     allocations (as xorec_gpu_cmp_bm.cpp:6-18 does); the deleter travels
//     with the pointer.
// A CPU-side plugin therefore overrides setup / encode / decode only
// (tests/host/plugin_defaults.cpp); the HIP plugin also overrides the three
// defaults because its buffers live in HBM.
//
// Differences from the reference, both for reproducibility: erasure sets and
// payloads come from explicit seeds (m_seed, bumped per setup() round through
// m_round) instead of the wall clock (utils.cpp:17-32, 100-127).
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>

#include "bm_config.hpp"

namespace xec {

using BufferDeleter = void (*)(uint8_t*);
using Buffer = std::unique_ptr<uint8_t[], BufferDeleter>;

// 64-B aligned host buffer (the reference's make_unique_aligned,
// utils.hpp; XOREC_ALIGNMENT); null on failure or when bytes == 0.
Buffer make_host_buffer(size_t bytes) noexcept;

class AbstractBenchmark {
 public:
  virtual ~AbstractBenchmark() noexcept = default;
  virtual void setup() noexcept = 0;
  virtual int encode() noexcept = 0;
  virtual int decode() noexcept = 0;
  virtual void simulate_data_loss() noexcept;
  virtual bool check_for_corruption() const noexcept;

 protected:
  explicit AbstractBenchmark(const BenchmarkConfig& config) noexcept;
  virtual void m_write_data_buffer() noexcept;

  // seed of block b of the current round's payload / stripe c's erasure draw
  uint64_t round_seed(uint64_t index) const noexcept { return m_seed + (m_round << 32) + index; }

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

  uint64_t m_seed;       // config.seed
  uint64_t m_round = 0;  // incremented by a plugin's setup(): fresh payload per iteration

  Buffer m_data_buf;      // S * k * bs
  Buffer m_parity_buf;    // S * m * bs
  Buffer m_block_bitmap;  // S * (k + m), 1 = present, 0 = lost
};

}  // namespace xec
