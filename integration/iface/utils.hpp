// utils.hpp -- this repository's restatement of the reference's
// src/utils/utils.hpp as the plugin interface uses it: the PCG32 generator,
// the validation payload, the erasure draw, throw_error and the owning
// buffer type every AbstractBenchmark buffer has (DeleterFunc /
// make_unique_aligned).  Declarations match utils.hpp:57-146; the bodies are
// utils.cpp here (restating utils.cpp:17-137).
//
// Left out: the reference's cuda_deleter / make_unique_cuda* templates
// (utils.hpp:124-180) -- CUDA runtime calls, which the MI355X plugins replace
// with integration/hip_buffers.hpp -- and the ECLimits of the other codecs.
#ifndef UTILS_HPP
#define UTILS_HPP

#define ENABLE_VALIDATION 1

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <memory>
#include <new>
#include <string>
#include <type_traits>

constexpr size_t ALIGNMENT = 64;
constexpr size_t RANDOM_SEED = 1896;
constexpr size_t MIN_DATA_BLOCK_SIZE = 2;

// PCG32 (utils.hpp:57-64; https://www.pcg-random.org/)
class PCGRandom {
 private:
  uint64_t state;
  uint64_t inc;

 public:
  PCGRandom(uint64_t seed, uint64_t seq);
  uint32_t next();
};

// Random payload from byte 8, the block length at 4 and a rotate-add checksum
// at 0 (blocks under 16 bytes: one repeated byte), seeded from the wall clock
// in milliseconds as the reference does; 0 on success, -1 if bytes < 2.
int write_validation_pattern(uint8_t* block_ptr, size_t bytes);

// True iff the block still carries the payload write_validation_pattern wrote.
bool validate_block(const uint8_t* block_ptr, size_t bytes);

// Marks num_lost_blocks of one stripe's bitmap 0, at most one per XOR-EC
// parity class (so the set is recoverable), drawn from the wall clock; prints
// and exits if num_lost_blocks > num_parity_blocks.
void select_lost_blocks(size_t num_data_blocks, size_t num_parity_blocks, size_t num_lost_blocks,
                        uint8_t* block_bitmap);

[[noreturn]] void throw_error(const std::string& message);

std::string to_lower(std::string str);

template <typename T>
using DeleterFunc = void (*)(T*);

template <typename T>
void mm_deleter(T* ptr) {
  std::free(ptr);
}

// ALIGNMENT-byte aligned, owning; throws std::bad_alloc on failure.
template <typename T>
std::unique_ptr<T[], DeleterFunc<T>> make_unique_aligned(size_t count = 1) {
  static_assert(std::is_trivially_destructible_v<T>, "Type must be trivially destructible");
  size_t bytes = count * sizeof(T);
  bytes = (bytes + ALIGNMENT - 1) / ALIGNMENT * ALIGNMENT;  // aligned_alloc wants a multiple
  void* mem = std::aligned_alloc(ALIGNMENT, bytes ? bytes : ALIGNMENT);
  if (mem == nullptr) throw std::bad_alloc();
  return std::unique_ptr<T[], DeleterFunc<T>>(static_cast<T*>(mem), mm_deleter<T>);
}

#endif  // UTILS_HPP
