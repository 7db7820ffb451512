// ThreadSanitizer test of integration/shard_pool.hpp (the multi-device plugin's
// per-shard decode threads): every run() calls fn(i) exactly once per shard,
// concurrently, and returns only after all of them; many back-to-back runs,
// pool sizes 1..9, construction and destruction with idle workers; and the
// Rendezvous decode() uses inside one run: every call gets the AND of all
// calls' flags, after all have arrived.
#include <atomic>
#include <cstdio>
#include <vector>

#include "shard_pool.hpp"

int main() {
  for (size_t n = 1; n <= 9; ++n) {
    xec_hip::ShardPool pool(n);
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
  for (size_t n = 1; n <= 9; ++n) {
    xec_hip::ShardPool pool(n);
    for (int round = 0; round < 500; ++round) {
      const size_t bad = static_cast<size_t>(round) % (n + 3);  // >= n: nobody fails
      xec_hip::Rendezvous rv(n);
      std::vector<int> before(n, 0), verdict(n, -1);  // plain ints, as above
      std::atomic<size_t> arrived{0};
      pool.run([&](size_t i) {
        before[i] = 1;
        arrived.fetch_add(1);
        const bool all = rv.arrive(i != bad);
        if (arrived.load() != n) verdict[i] = 2;  // returned before everyone arrived
        else verdict[i] = all ? 1 : 0;
      });
      for (size_t i = 0; i < n; ++i)
        if (before[i] != 1 || verdict[i] != (bad >= n ? 1 : 0)) {
          std::printf("rendezvous n=%zu round %d shard %zu: verdict %d\n", n, round, i, verdict[i]);
          return 1;
        }
    }
  }
  { xec_hip::ShardPool idle(4); }  // destroyed without a run
  std::printf("shard_pool ok\n");
  return 0;
}
