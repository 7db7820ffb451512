// ec_utils.cpp -- see ec_utils.hpp.
#include "ec_utils.hpp"

#include <algorithm>
#include <cstring>
#include <vector>

namespace xec {

namespace {
inline uint32_t rotl3(uint32_t x) { return (x << 3) | (x >> 29); }
}  // namespace

int write_validation_block(uint8_t* block, size_t bytes, uint64_t seed) {
  if (bytes < 2) return -1;
  Pcg32 rng(kRandomSeed + seed, 1);
  if (bytes < 16) {
    std::fill(block, block + bytes, static_cast<uint8_t>(rng.next()));
    return 0;
  }
  const uint32_t len = static_cast<uint32_t>(bytes);
  uint32_t crc = len;
  for (size_t i = 8; i < bytes; ++i) {
    const uint8_t v = static_cast<uint8_t>(rng.next());
    block[i] = v;
    crc = rotl3(crc) + v;
  }
  std::memcpy(block + 4, &len, sizeof len);
  std::memcpy(block, &crc, sizeof crc);
  return 0;
}

bool validate_block(const uint8_t* block, size_t bytes) {
  if (bytes < 2) return false;
  if (bytes < 16) return std::all_of(block + 1, block + bytes, [&](uint8_t b) { return b == block[0]; });
  uint32_t len = 0, stored = 0;
  std::memcpy(&len, block + 4, sizeof len);
  if (len != static_cast<uint32_t>(bytes)) return false;
  uint32_t crc = len;
  for (size_t i = 8; i < bytes; ++i) crc = rotl3(crc) + block[i];
  std::memcpy(&stored, block, sizeof stored);
  return stored == crc;
}

int select_lost_blocks(size_t k, size_t m, size_t lost, uint8_t* bitmap, uint64_t seed) {
  if (lost == 0) return 0;
  if (lost > m) return -1;
  std::vector<uint32_t> candidates(k + m);
  for (size_t i = 0; i < candidates.size(); ++i) candidates[i] = static_cast<uint32_t>(i);
  Pcg32 rng(kRandomSeed + seed, 1);
  for (size_t n = 0; n < lost; ++n) {
    const uint32_t idx = candidates[rng.next() % candidates.size()];
    bitmap[idx] = 0;
    const uint32_t cls = static_cast<uint32_t>(idx % m);
    candidates.erase(std::remove_if(candidates.begin(), candidates.end(),
                                    [&](uint32_t c) { return c % m == cls; }),
                     candidates.end());
  }
  return 0;
}

}  // namespace xec
