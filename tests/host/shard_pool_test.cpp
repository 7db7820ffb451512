// ThreadSanitizer test of host/shard_pool.hpp (the multi-device plugin's
// per-shard decode threads): every run() calls fn(i) exactly once per shard,
// concurrently, and returns only after all of them; many back-to-back runs,
// pool sizes 1..9, construction and destruction with idle workers.
#include <atomic>
#include <cstdio>
#include <vector>

#include "shard_pool.hpp"

int main() {
  for (size_t n = 1; n <= 9; ++n) {
    xec::ShardPool pool(n);
    std::vector<int> hits(n, 0);  // plain ints: TSan flags any unordered access
    for (int round = 0; round < 2000; ++round) {
      std::atomic<size_t> running{0};
      pool.run([&](size_t i) {
        running.fetch_add(1);
        hits[i] += 1;
      });
      if (running.load() != n) {
        std::printf("round %d: %zu of %zu shards ran\n", round, running.load(), n);
        return 1;
      }
      for (size_t i = 0; i < n; ++i)
        if (hits[i] != round + 1) {
          std::printf("shard %zu ran %d times after %d rounds\n", i, hits[i], round + 1);
          return 1;
        }
    }
  }
  { xec::ShardPool idle(4); }  // destroyed without a run
  std::printf("shard_pool ok\n");
  return 0;
}
