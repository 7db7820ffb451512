// ref_driver.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A command-line driver around the reference's OWN, unmodified CPU XOR-EC
// sources (/root/reference/src/xorec/xorec.cpp, xorec_utils.cpp,
// src/utils/utils.cpp), compiled by oracle/Makefile into oracle/_ref/.  It is
// used in this container to pin the C restatement (oracle/xorec_oracle.c) and
// to generate tests/golden/ fixtures (tests/golden/make_golden.py).  Nothing
// here is product code and nothing from the reference is copied into the repo:
// this file only calls the reference's public functions
// (xorec_init / xorec_encode / xorec_decode, xorec.hpp:39-79;
//  validate_block, utils.hpp:73).
//
// Commands (all output on stdout, one "key value" per line):
//   enc K M BS S SEED VERSION [PARITY_OUT]
//   dec K M BS S SEED VERSION MODE [ARG]     MODE: single7 | pattern FILE | none
//   chk K M BS DATA_MISALIGN PARITY_MISALIGN
//   val BS FILE                               validate_block per BS-byte block
//   bench K M BS S VERSION THREADS SECONDS    time the reference CPU path (bench.py's
//                                             cpu_baseline, kind "reference")
#include "xorec.hpp"
#include "utils.hpp"

#include <omp.h>
#include <sys/mman.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

uint64_t splitmix_at(uint64_t seed, uint64_t n) {
  uint64_t z = seed + (n + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t fnv(const uint8_t* p, size_t n, uint64_t h = 0xcbf29ce484222325ull) {
  for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 0x100000001b3ull; }
  return h;
}

// 64-B aligned (the reference's ALIGNMENT, utils.hpp:25).  With REF_HUGEPAGES=1
// the buffer is 2 MiB aligned and madvise(MADV_HUGEPAGE)d, as numpy does for the
// oracle's buffers, so both CPU baselines see the same page size.
uint8_t* alloc64(size_t n) {
  const char* hp = std::getenv("REF_HUGEPAGES");
  const bool huge = hp && hp[0] == '1' && n >= (4u << 20);
  const size_t align = huge ? (2u << 20) : 64;
  size_t r = (n + align - 1) / align * align + align;
  auto* p = static_cast<uint8_t*>(std::aligned_alloc(align, r));
  if (huge) madvise(p, r, MADV_HUGEPAGE);
  std::memset(p, 0, r);
  return p;
}

void fill(uint8_t* d, size_t S, size_t stripe, uint64_t seed) {
  for (size_t c = 0; c < S; ++c) {
    auto* w = reinterpret_cast<uint64_t*>(d + c * stripe);
    for (size_t n = 0; n < stripe / 8; ++n) w[n] = splitmix_at(seed + c, n);
  }
}

XorecVersion ver(int v) { return static_cast<XorecVersion>(v); }

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) { std::fprintf(stderr, "usage: see header\n"); return 2; }
  xorec_init(4096);  // size COMPLETE_DATA_BITMAP once for every k used here
  std::string cmd = argv[1];

  if (cmd == "enc" || cmd == "dec") {
    size_t k = std::strtoull(argv[2], nullptr, 0), m = std::strtoull(argv[3], nullptr, 0);
    size_t bs = std::strtoull(argv[4], nullptr, 0), S = std::strtoull(argv[5], nullptr, 0);
    uint64_t seed = std::strtoull(argv[6], nullptr, 0);
    int v = std::atoi(argv[7]);
    uint8_t* data = alloc64(S * k * bs);
    uint8_t* parity = alloc64(S * m * bs);
    fill(data, S, k * bs, seed);
    int enc_fail = 0;
    for (size_t c = 0; c < S; ++c)
      if (xorec_encode(data + c * k * bs, parity + c * m * bs, bs, k, m, ver(v)) != XorecResult::Success)
        enc_fail++;
    std::printf("enc_fail %d\nparity_fnv %016llx\n", enc_fail,
                (unsigned long long)fnv(parity, S * m * bs));
    if (cmd == "enc") {
      if (argc > 8) {
        FILE* f = std::fopen(argv[8], "wb");
        std::fwrite(parity, 1, S * m * bs, f);
        std::fclose(f);
      }
      return 0;
    }
    std::string mode = argv[8];
    std::vector<uint8_t> bitmap(S * (k + m), 1);
    if (mode == "single7") {
      for (size_t c = 0; c < S; ++c) bitmap[c * (k + m) + (7 * c) % k] = 0;
    } else if (mode == "pattern") {
      FILE* f = std::fopen(argv[9], "rb");
      size_t got = std::fread(bitmap.data(), 1, bitmap.size(), f);
      std::fclose(f);
      if (got != bitmap.size()) { std::fprintf(stderr, "short pattern\n"); return 2; }
    }
    uint64_t data_fnv_before = fnv(data, S * k * bs);
    // erase: lost blocks zeroed, as AbstractBenchmark::simulate_data_loss does
    for (size_t c = 0; c < S; ++c)
      for (size_t i = 0; i < k + m; ++i)
        if (!bitmap[c * (k + m) + i]) {
          uint8_t* blk = i < k ? data + c * k * bs + i * bs : parity + c * m * bs + (i - k) * bs;
          std::memset(blk, 0, bs);
        }
    uint64_t parity_fnv_erased = fnv(parity, S * m * bs);
    std::string codes;
    for (size_t c = 0; c < S; ++c) {
      XorecResult r = xorec_decode(data + c * k * bs, parity + c * m * bs, bs, k, m,
                                   bitmap.data() + c * (k + m), ver(v));
      codes += static_cast<char>('0' + static_cast<int>(r));
    }
    std::printf("data_fnv_before %016llx\n", (unsigned long long)data_fnv_before);
    std::printf("data_fnv_after %016llx\n", (unsigned long long)fnv(data, S * k * bs));
    std::printf("parity_fnv_erased %016llx\n", (unsigned long long)parity_fnv_erased);
    std::printf("parity_fnv_after %016llx\n", (unsigned long long)fnv(parity, S * m * bs));
    std::printf("codes %s\n", codes.c_str());
    return 0;
  }

  if (cmd == "chk") {
    size_t k = std::strtoull(argv[2], nullptr, 0), m = std::strtoull(argv[3], nullptr, 0);
    size_t bs = std::strtoull(argv[4], nullptr, 0);
    size_t dm = std::strtoull(argv[5], nullptr, 0), pm = std::strtoull(argv[6], nullptr, 0);
    size_t kk = k ? k : 1, mm = m ? m : 1;
    uint8_t* data = alloc64(kk * bs + 64);
    uint8_t* parity = alloc64(mm * bs + 64);
    std::vector<uint8_t> bitmap(kk + mm + 8, 1);
    bitmap[0] = 0;  // one lost data block so decode gets past require_recovery
    XorecResult e = xorec_encode(data + dm, parity + pm, bs, k, m, XorecVersion::Scalar);
    XorecResult d = xorec_decode(data + dm, parity + pm, bs, k, m, bitmap.data(), XorecVersion::Scalar);
    std::printf("encode %d\ndecode %d\n", static_cast<int>(e), static_cast<int>(d));
    return 0;
  }

  if (cmd == "bench") {
    // bench K M BS S VERSION THREADS SECONDS: the reference's CPU plugin loop
    // (XorecBenchmark::encode/decode, xorec_bm.cpp:27-58: omp parallel for
    // over stripes calling xorec_encode / xorec_decode), timed on the
    // reference's own xorec code; single erasure (7c) mod k per stripe.
    size_t k = std::strtoull(argv[2], nullptr, 0), m = std::strtoull(argv[3], nullptr, 0);
    size_t bs = std::strtoull(argv[4], nullptr, 0), S = std::strtoull(argv[5], nullptr, 0);
    int v = std::atoi(argv[6]), threads = std::atoi(argv[7]);
    double budget = std::atof(argv[8]);
    omp_set_num_threads(threads);
    uint8_t* data = alloc64(S * k * bs);
    uint8_t* parity = alloc64(S * m * bs);
#pragma omp parallel for schedule(static)
    for (long c = 0; c < (long)S; ++c) fill(data + c * k * bs, 1, k * bs, 1896 + c);
    std::vector<uint8_t> bitmap(S * (k + m), 1);
    for (size_t c = 0; c < S; ++c) bitmap[c * (k + m) + (7 * c) % k] = 0;
    int fail = 0, reps = 0;
    double t = 0;
    while (t < budget && reps < 100000) {
      double t0 = omp_get_wtime();
#pragma omp parallel for schedule(static) reduction(+ : fail)
      for (long c = 0; c < (long)S; ++c)
        fail += xorec_encode(data + c * k * bs, parity + c * m * bs, bs, k, m, ver(v)) !=
                XorecResult::Success;
#pragma omp parallel for schedule(static) reduction(+ : fail)
      for (long c = 0; c < (long)S; ++c)
        fail += xorec_decode(data + c * k * bs, parity + c * m * bs, bs, k, m,
                             bitmap.data() + c * (k + m), ver(v)) != XorecResult::Success;
      t += omp_get_wtime() - t0;
      ++reps;
    }
    std::printf("reps %d\nseconds %.6f\nfail %d\nparity_fnv %016llx\n", reps, t, fail,
                (unsigned long long)fnv(parity, S * m * bs));
    return 0;
  }

  if (cmd == "val") {
    size_t bs = std::strtoull(argv[2], nullptr, 0);
    FILE* f = std::fopen(argv[3], "rb");
    std::vector<uint8_t> blk(bs);
    std::string out;
    while (std::fread(blk.data(), 1, bs, f) == bs) out += validate_block(blk.data(), bs) ? '1' : '0';
    std::fclose(f);
    std::printf("valid %s\n", out.c_str());
    return 0;
  }
  std::fprintf(stderr, "unknown command %s\n", cmd.c_str());
  return 2;
}
