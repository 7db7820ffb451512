// ec_utils.hpp -- host utilities of the benchmark harness (product side).
//
// Behaviour follows the reference's src/utils/utils.cpp, with the wall-clock
// seeds replaced by explicit ones so every run is reproducible:
//   Pcg32                   PCGRandom                 utils.cpp:17-32
//   write_validation_block  write_validation_pattern  utils.cpp:35-69
//   validate_block          validate_block            utils.cpp:72-97
//   select_lost_blocks      select_lost_blocks        utils.cpp:100-127
#pragma once

#include <cstddef>
#include <cstdint>

namespace xec {

constexpr uint64_t kRandomSeed = 1896;  // RANDOM_SEED, utils.hpp:26

class Pcg32 {
 public:
  Pcg32(uint64_t seed, uint64_t seq) : state_(0), inc_((seq << 1u) | 1u) {
    next();
    state_ += seed;
    next();
  }
  uint32_t next() {
    uint64_t old = state_;
    state_ = old * 6364136223846793005ull + inc_;
    uint32_t xs = static_cast<uint32_t>(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = static_cast<uint32_t>(old >> 59u);
    return (xs >> rot) | (xs << ((0u - rot) & 31u));
  }

 private:
  uint64_t state_, inc_;
};

// Random payload from byte 8, u32 length at 4, u32 rotate-add checksum at 0
// (blocks < 16 B: one repeated random byte).  Returns 0, or -1 if bytes < 2.
int write_validation_block(uint8_t* block, size_t bytes, uint64_t seed);
bool validate_block(const uint8_t* block, size_t bytes);

// Marks `lost` blocks of one stripe's (k+m)-byte bitmap as 0, at most one per
// parity class (so the set is always recoverable).  Returns -1 if lost > m
// (where the reference prints and exits).
int select_lost_blocks(size_t k, size_t m, size_t lost, uint8_t* bitmap, uint64_t seed);

}  // namespace xec
