// iface_utils.cpp -- the restated interface utilities (integration/iface/utils.cpp)
// against the oracle's restatement of the reference's (oracle/xorec_oracle.c,
// pinned to the reference's own sources by tests/test_oracle.py):
//   PCGRandom         == xo_pcg over many seeds and streams (utils.cpp:17-32)
//   validate_block    accepts the oracle's payloads, rejects a flipped byte and
//                     a wrong length (utils.cpp:72-97)
//   write_validation_pattern (wall clock) writes payloads the oracle's
//                     validate accepts (utils.cpp:35-69)
//   select_lost_blocks (wall clock) marks exactly `lost` blocks, one per parity
//                     class (utils.cpp:100-127)
// CPU only (tests/test_plugin_interface.py).  Prints "iface_utils ok".
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "utils.hpp"
#include "xorec_oracle.h"

namespace {

int failures = 0;
void expect(bool ok, const std::string& what) {
  if (!ok) {
    std::printf("FAIL %s\n", what.c_str());
    ++failures;
  }
}

}  // namespace

int main() {
  for (uint64_t seed : {0ull, 1ull, 1896ull, 1ull << 40, 0xFFFFFFFFFFFFFFFFull})
    for (uint64_t seq : {0ull, 1ull, 7ull}) {
      PCGRandom a(seed, seq);
      xo_pcg b;
      xo_pcg_init(&b, seed, seq);
      bool same = true;
      for (int i = 0; i < 1000; ++i) same = same && a.next() == xo_pcg_next(&b);
      expect(same, "PCGRandom == xo_pcg, seed " + std::to_string(seed));
    }
  for (size_t bs : {2ul, 3ul, 15ul, 16ul, 17ul, 256ul, 1000ul, 4096ul, 65536ul}) {
    std::vector<uint8_t> blk(bs);
    for (uint64_t seed : {0ull, 5ull, 1ull << 33}) {
      xo_write_validation_pattern(blk.data(), bs, seed);
      expect(validate_block(blk.data(), bs), "validate_block(oracle payload) bs " + std::to_string(bs));
      if (bs >= 16) {
        blk[bs / 2 + 4] ^= 0x10;
        expect(!validate_block(blk.data(), bs), "flipped byte rejected bs " + std::to_string(bs));
        blk[bs / 2 + 4] ^= 0x10;
        expect(!validate_block(blk.data(), bs - 1), "wrong length rejected bs " + std::to_string(bs));
      } else {
        blk[bs - 1] ^= 1;
        expect(!validate_block(blk.data(), bs), "small block: a differing byte rejected");
      }
    }
    expect(write_validation_pattern(blk.data(), bs) == 0, "write_validation_pattern rc");
    expect(xo_validate_block(blk.data(), bs) != 0,
           "oracle validates write_validation_pattern bs " + std::to_string(bs));
  }
  std::vector<uint8_t> one(1);
  expect(write_validation_pattern(one.data(), 1) != 0, "bytes < 2 refused");
  for (size_t k : {4ul, 16ul, 32ul})
    for (size_t m : {1ul, 2ul, 4ul, 8ul}) {
      if (k % m) continue;
      for (size_t lost = 0; lost <= m; ++lost) {
        std::vector<uint8_t> bm(k + m, 1);
        select_lost_blocks(k, m, lost, bm.data());
        std::vector<int> cls(m, 0);
        size_t zeros = 0;
        bool one_per_class = true;
        for (size_t i = 0; i < k + m; ++i)
          if (!bm[i]) {
            ++zeros;
            one_per_class = one_per_class && cls[i % m]++ == 0;
          }
        expect(zeros == lost && one_per_class && xo_is_recoverable(k, m, bm.data()),
               "select_lost_blocks k " + std::to_string(k) + " m " + std::to_string(m));
      }
    }
  if (failures == 0) std::printf("iface_utils ok\n");
  return failures ? 1 : 0;
}
