// drop_in.cpp -- the drop-in plugins themselves (integration/xorec_hip_bm.cpp,
// integration/xorec_hip_multi_bm.cpp, built into libxec_plugin.so over this
// repo's restatement of the reference's interface) driven through
// AbstractBenchmark& exactly as the reference's BM_generic drives a plugin
// (src/benchmark/abstract_runner.hpp:97-121: setup | encode |
// simulate_data_loss | decode | check_for_corruption), with every step
// checked against the oracle (oracle/xorec_oracle.c, test infrastructure):
//   after encode      parity == the oracle's encode of the batch's data
//                     (xorec.cpp:24-59); seeded: the data == the oracle's
//                     validation payload (utils.cpp:35-69, explicit seed)
//   after the losses  each stripe lost `lost` blocks, one per parity class
//                     (select_lost_blocks, utils.cpp:100-127; seeded: the
//                     oracle's draw, same seed), those blocks are zero and
//                     every other byte is untouched
//   after decode      decode() == 0, the data is the pre-loss data byte for
//                     byte, parity untouched, and check_for_corruption() holds
//
//   drop_in single|multi MESSAGE BLOCK TOTAL DATA LOST [SEED] [ITERATIONS]
//
// No SEED: the one-argument constructor, i.e. the reference's registration
// and its wall-clock payloads / erasure draws.  multi: the devices come from
// XEC_DEVICES (or the options with SEED).  Prints "drop_in ok" on success.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include "xec_plugin_options.hpp"
#include "xorec_hip_bm.hpp"
#include "xorec_hip_multi_bm.hpp"
#include "xorec_oracle.h"

namespace {

// 64-B aligned host memory: the oracle checks XOREC_ALIGNMENT as the
// reference does (xorec_utils.hpp:61-86)
template <class T>
struct Aligned64 {
  using value_type = T;
  Aligned64() = default;
  template <class U>
  Aligned64(const Aligned64<U>&) {}
  T* allocate(size_t n) {
    void* p = std::aligned_alloc(64, (n * sizeof(T) + 63) / 64 * 64);
    if (p == nullptr) throw std::bad_alloc();
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_t) { std::free(p); }
  template <class U>
  bool operator==(const Aligned64<U>&) const { return true; }
  template <class U>
  bool operator!=(const Aligned64<U>&) const { return false; }
};
using Bytes = std::vector<uint8_t, Aligned64<uint8_t>>;

template <class P>
class Probe : public P {
 public:
  using P::P;
  size_t S() const { return this->m_chunks; }
  const uint8_t* bitmap() const { return this->m_block_bitmap.get(); }
  bool read(Bytes& d, Bytes& p) const {
    d.assign(this->m_chunks * this->m_chunk_data_size, 0);
    p.assign(this->m_chunks * this->m_chunk_parity_size, 0);
    if constexpr (std::is_same_v<P, XorecBenchmarkHipMulti>) {
      for (size_t i = 0; i < this->num_shards(); ++i)
        if (!this->read_shard(i, d.data() + this->shard_first(i) * this->m_chunk_data_size,
                              p.data() + this->shard_first(i) * this->m_chunk_parity_size))
          return false;
      return true;
    } else {
      return hipDeviceSynchronize() == hipSuccess &&
             hipMemcpy(d.data(), this->m_data_buf.get(), d.size(), hipMemcpyDeviceToHost) ==
                 hipSuccess &&
             hipMemcpy(p.data(), this->m_parity_buf.get(), p.size(), hipMemcpyDeviceToHost) ==
                 hipSuccess;
    }
  }
};

int fail(const char* what, int iter) {
  std::printf("drop_in FAILED: %s (iteration %d)\n", what, iter);
  std::fflush(stdout);
  std::_Exit(1);
}

template <class P>
int run(const BenchmarkConfig& c, bool seeded, uint64_t seed, int iterations) {
  const size_t k = std::get<1>(c.ec_params), m = std::get<0>(c.ec_params) - k, bs = c.block_size;
  const size_t tot = k + m;
  std::unique_ptr<Probe<P>> probe;
  if (seeded) {
    XecPluginOptions opt;
    opt.seeded = true;
    opt.seed = seed;
    probe = std::make_unique<Probe<P>>(c, opt);
  } else {
    probe = std::make_unique<Probe<P>>(c);  // the reference's registration
  }
  AbstractBenchmark& bench = *probe;  // BM_generic sees the interface only
  const size_t S = probe->S();
  Bytes d0, p0, d1, p1, d2, p2, want(S * m * bs);
  for (int it = 1; it <= iterations; ++it) {
    bench.setup();
    if (bench.encode() != 0) return fail("encode() != 0", it);
    if (!probe->read(d0, p0)) return fail("read after encode", it);
    if (seeded) {  // the payload: block b of round r from seed + (r << 32) + b
      std::vector<uint8_t> blk(bs);
      for (size_t b = 0; b < S * k; ++b) {
        xo_write_validation_pattern(blk.data(), bs, seed + (uint64_t(it) << 32) + b);
        if (std::memcmp(blk.data(), d0.data() + b * bs, bs) != 0)
          return fail("seeded payload != oracle's write_validation_pattern", it);
      }
    }
    if (xo_encode_batch(d0.data(), want.data(), S, bs, k, m, 0) != XO_SUCCESS)
      return fail("oracle encode", it);
    if (want != p0) return fail("parity != oracle encode", it);
    bench.simulate_data_loss();
    if (!probe->read(d1, p1)) return fail("read after simulate_data_loss", it);
    const uint8_t* bm = probe->bitmap();
    for (size_t s = 0; s < S; ++s) {
      const uint8_t* row = bm + s * tot;
      std::vector<int> cls(m, 0);
      size_t zeros = 0;
      for (size_t i = 0; i < tot; ++i) {
        const uint8_t* blk = i < k ? d1.data() + (s * k + i) * bs : p1.data() + (s * m + i - k) * bs;
        const uint8_t* was = i < k ? d0.data() + (s * k + i) * bs : p0.data() + (s * m + i - k) * bs;
        if (row[i]) {
          if (std::memcmp(blk, was, bs) != 0) return fail("a surviving block changed", it);
          continue;
        }
        ++zeros;
        if (cls[i % m]++) return fail("two losses in one parity class", it);
        for (size_t x = 0; x < bs; ++x)
          if (blk[x]) return fail("a lost block is not zero", it);
      }
      if (zeros != c.num_lost_blocks) return fail("wrong loss count", it);
      if (seeded) {
        std::vector<uint8_t> w(tot, 1);
        xo_select_lost_blocks(k, m, c.num_lost_blocks, w.data(),
                              seed + (uint64_t(it) << 32) + s);
        if (std::memcmp(w.data(), row, tot) != 0) return fail("erasure draw != oracle's", it);
      }
    }
    if (bench.decode() != 0) return fail("decode() != 0", it);
    if (!probe->read(d2, p2)) return fail("read after decode", it);
    if (d2 != d0) return fail("rebuilt data != pre-loss data", it);
    if (p2 != p1) return fail("decode touched the parity", it);
    if (!bench.check_for_corruption()) return fail("check_for_corruption() false", it);
  }
  std::printf("drop_in ok S=%zu k=%zu m=%zu bs=%zu lost=%zu seeded=%d iterations=%d\n", S, k, m,
              bs, c.num_lost_blocks, seeded ? 1 : 0, iterations);
  return 0;
}

size_t num(const char* s) {
  char* end = nullptr;
  unsigned long long v = std::strtoull(s, &end, 0);
  if (*end == 'K') v <<= 10;
  if (*end == 'M') v <<= 20;
  if (*end == 'G') v <<= 30;
  return static_cast<size_t>(v);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 7) {
    std::fprintf(stderr, "usage: drop_in single|multi MESSAGE BLOCK TOTAL DATA LOST [SEED] [ITERS]\n");
    return 2;
  }
  BenchmarkConfig c{};
  c.message_size = num(argv[2]);
  c.block_size = num(argv[3]);
  c.ec_params = ECTuple(num(argv[4]), num(argv[5]));
  c.num_lost_blocks = num(argv[6]);
  c.num_cpu_threads = 1;
  c.num_iterations = 1;
  c.num_warmup_iterations = 0;
  c.gpu_computation = true;
  const bool seeded = argc > 7 && std::string(argv[7]) != "-";
  const uint64_t seed = seeded ? num(argv[7]) : 0;
  const int iters = argc > 8 ? std::atoi(argv[8]) : 2;
  int rc = 0;
  try {
    rc = std::string(argv[1]) == "multi" ? run<XorecBenchmarkHipMulti>(c, seeded, seed, iters)
                                         : run<XorecBenchmarkHip>(c, seeded, seed, iters);
  } catch (const std::exception& e) {
    std::printf("drop_in FAILED: %s\n", e.what());
    rc = 3;
  }
  std::fflush(stdout);
  std::_Exit(rc);  // as multi_equiv.cpp: skip the HIP runtime's static teardown
}
