// utils.cpp -- see utils.hpp.  Restates src/utils/utils.cpp:17-137 (the
// behaviour, including the wall-clock seeds: two blocks written in the same
// millisecond carry the same payload, as in the reference).
#include "utils.hpp"

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <vector>

namespace {

uint64_t clock_ms() {
  return static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::milliseconds>(
                                   std::chrono::system_clock::now().time_since_epoch())
                                   .count());
}

inline uint32_t spread(uint32_t crc) { return (crc << 3) | (crc >> 29); }

}  // namespace

// utils.cpp:17-32
PCGRandom::PCGRandom(uint64_t seed, uint64_t seq) : state(0), inc((seq << 1) | 1) {
  next();
  state += seed;
  next();
}

uint32_t PCGRandom::next() {
  const uint64_t old = state;
  state = old * 6364136223846793005ull + inc;
  const uint32_t x = static_cast<uint32_t>(((old >> 18u) ^ old) >> 27u);
  const uint32_t r = static_cast<uint32_t>(old >> 59u);
  return (x >> r) | (x << ((0u - r) & 31u));
}

// utils.cpp:35-69
int write_validation_pattern(uint8_t* block_ptr, size_t bytes) {
  if (bytes < 2) return -1;
  PCGRandom rng(RANDOM_SEED + clock_ms(), 1);
  if (bytes < 16) {
    std::memset(block_ptr, static_cast<uint8_t>(rng.next()), bytes);
    return 0;
  }
  const uint32_t len = static_cast<uint32_t>(bytes);
  uint32_t crc = len;
  for (size_t i = 8; i < bytes; ++i) {
    const uint8_t v = static_cast<uint8_t>(rng.next());
    block_ptr[i] = v;
    crc = spread(crc) + v;
  }
  std::memcpy(block_ptr + 4, &len, sizeof len);
  std::memcpy(block_ptr, &crc, sizeof crc);
  return 0;
}

// utils.cpp:72-97
bool validate_block(const uint8_t* block_ptr, size_t bytes) {
  if (bytes < 2) return false;
  if (bytes < 16)
    return std::all_of(block_ptr + 1, block_ptr + bytes,
                       [first = block_ptr[0]](uint8_t b) { return b == first; });
  uint32_t len = 0, stored = 0;
  std::memcpy(&len, block_ptr + 4, sizeof len);
  if (len != static_cast<uint32_t>(bytes)) return false;
  uint32_t crc = len;
  for (size_t i = 8; i < bytes; ++i) crc = spread(crc) + block_ptr[i];
  std::memcpy(&stored, block_ptr, sizeof stored);
  return stored == crc;
}

// utils.cpp:100-127
void select_lost_blocks(size_t num_data_blocks, size_t num_parity_blocks, size_t num_lost_blocks,
                        uint8_t* block_bitmap) {
  if (num_lost_blocks == 0) return;
  if (num_lost_blocks > num_parity_blocks) {
    std::fprintf(stderr,
                 "select_lost_blocks: Number of lost blocks must be less than or equal to the "
                 "number of recovery blocks\n");
    std::exit(EXIT_SUCCESS);
  }
  PCGRandom rng(RANDOM_SEED + clock_ms(), 1);
  std::vector<uint32_t> eligible(num_data_blocks + num_parity_blocks);
  for (size_t i = 0; i < eligible.size(); ++i) eligible[i] = static_cast<uint32_t>(i);
  for (size_t d = 0; d < num_lost_blocks; ++d) {
    const uint32_t lost = eligible[rng.next() % eligible.size()];
    block_bitmap[lost] = 0;
    const size_t cls = lost % num_parity_blocks;
    eligible.erase(std::remove_if(eligible.begin(), eligible.end(),
                                  [&](uint32_t b) { return b % num_parity_blocks == cls; }),
                   eligible.end());
  }
}

[[noreturn]] void throw_error(const std::string& message) { throw std::runtime_error(message); }

std::string to_lower(std::string str) {
  for (char& c : str) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return str;
}
