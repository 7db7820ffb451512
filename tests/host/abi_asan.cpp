// abi_asan.cpp -- the C ABI's host code under AddressSanitizer on the GPU box
// (built by tests/host/Makefile as bin/asan_abi: csrc/xec_api.cpp,
// xec_scan.cpp and xec_pipeline.cpp compiled in with host-only ASan, the
// kernels as usual; run by tests/test_plugin_harness.py).
//
// Every host buffer the library reads or writes -- bitmaps, per-stripe codes,
// the pipeline's host batch -- is an exact-size new[] allocation, so an
// over- or under-read in the scans, the work-list staging, the kernel-argument
// lists or the pipeline's run merging is an ASan report.  Results are checked
// too: parity against a host XOR of each class, decodes (every tiling,
// per-stripe, pipeline) against the original bytes, or untouched when a stripe
// is unrecoverable.  Prints "abi_asan ok".
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "xec.h"

namespace {

int fail(int code, const char* what, int c) {
  std::printf("case %d: %s (%d)\n", c, what, code);
  return code;
}

int one_case(std::mt19937_64& rng, int c) {
  const size_t ms[] = {1, 1, 2, 3, 4, 8};
  const size_t m = ms[rng() % 6];
  const size_t k = m * (1 + rng() % (40 / m));
  const size_t bs = 256 * (1 + rng() % 64);
  const size_t S = 1 + rng() % 300;
  const size_t row = k + m, nd = S * k * bs, np = S * m * bs;
  uint8_t *d = nullptr, *p = nullptr, *dbm = nullptr;
  if (hipMalloc(&d, nd) || hipMalloc(&p, np) || hipMalloc(&dbm, S * row)) return 90;
  if (xec_fill_splitmix64(d, S, k * bs, 700 + c, nullptr) || xec_encode(d, p, S, bs, k, m, nullptr) ||
      hipDeviceSynchronize())
    return fail(1, "encode", c);
  std::vector<uint8_t> hd(nd), hp(np), ref(np, 0);
  if (hipMemcpy(hd.data(), d, nd, hipMemcpyDeviceToHost) || hipMemcpy(hp.data(), p, np, hipMemcpyDeviceToHost))
    return 91;
  for (size_t s = 0; s < S; ++s)
    for (size_t i = 0; i < k; ++i) {
      const uint8_t* src = &hd[(s * k + i) * bs];
      uint8_t* dst = &ref[(s * m + i % m) * bs];
      for (size_t b = 0; b < bs; ++b) dst[b] ^= src[b];
    }
  if (hp != ref) return fail(2, "parity", c);
  // loss pattern: per stripe 0..m data blocks in distinct classes; sometimes
  // a lost parity; one case in 5 has an unrecoverable stripe
  uint8_t* bm = new uint8_t[S * row];  // exact size: ASan sees any overread
  std::memset(bm, 1, S * row);
  bool recoverable = true;
  size_t bad_stripe = S;
  const int sparse = c % 3 == 0;
  for (size_t s = 0; s < S; ++s) {
    if (sparse && rng() % 9) continue;
    const size_t lost = rng() % (m + 1);
    std::vector<size_t> cls(m);
    for (size_t j = 0; j < m; ++j) cls[j] = j;
    std::shuffle(cls.begin(), cls.end(), rng);
    for (size_t q = 0; q < lost; ++q) bm[s * row + cls[q] + m * (rng() % (k / m))] = 0;
    for (size_t q = lost; q < m; ++q)
      if (rng() % 4 == 0) bm[s * row + k + cls[q]] = 0;  // parity of a class without data loss
  }
  if (c % 5 == 4) {
    const size_t s = rng() % S;
    std::memset(bm + s * row, 1, row);
    bm[s * row] = 0;
    bm[s * row + k] = 0;
    recoverable = false;
    bad_stripe = s;
  }
  std::vector<uint8_t> erased = hd;
  for (size_t s = 0; s < S; ++s)
    for (size_t i = 0; i < k; ++i)
      if (!bm[s * row + i]) std::memset(&erased[(s * k + i) * bs], 0, bs);
  std::vector<uint8_t> got(nd);
  int rc = 0;
  // xec_decode under every tiling, then the per-stripe decode
  for (int tiling = 0; tiling <= 4 && rc == 0; ++tiling) {
    if (hipMemcpy(d, erased.data(), nd, hipMemcpyHostToDevice)) return 92;
    xec_status st;
    if (tiling < 4) {
      xec_set_decode_tiling(tiling);
      st = xec_decode(d, p, S, bs, k, m, bm, dbm, nullptr);
      xec_set_decode_tiling(0);
    } else {
      uint8_t* codes = new uint8_t[S];
      st = xec_decode_per_stripe(d, p, S, bs, k, m, bm, dbm, codes, nullptr);
      delete[] codes;
    }
    if (hipDeviceSynchronize() || hipMemcpy(got.data(), d, nd, hipMemcpyDeviceToHost)) return 93;
    if (tiling < 4) {
      if (st != (recoverable ? XEC_SUCCESS : XEC_DECODE_FAILURE)) rc = fail(3, "decode status", c);
      else if (got != (recoverable ? hd : erased)) rc = fail(4, "decode bytes", c);
    } else if (st != (recoverable ? XEC_SUCCESS : XEC_DECODE_FAILURE)) {
      rc = fail(5, "per-stripe status", c);
    } else {  // recoverable stripes rebuilt, the failing one left as erased
      std::vector<uint8_t> want = hd;
      if (bad_stripe < S)
        std::memcpy(&want[bad_stripe * k * bs], &erased[bad_stripe * k * bs], k * bs);
      if (got != want) rc = fail(10, "per-stripe bytes", c);
    }
  }
  // the host-in / host-out pipeline over exact-size pageable host buffers
  if (rc == 0) {
    xec_pipeline* pl = nullptr;
    if (xec_pipeline_create(&pl, 1 + rng() % 9, bs, k, m, 1 + (int)(rng() % 3))) return fail(6, "pipeline create", c);
    uint8_t* h_data = new uint8_t[nd];
    uint8_t* h_par = new uint8_t[np];
    std::memcpy(h_data, hd.data(), nd);
    std::memset(h_par, 0, np);
    if (xec_pipeline_encode(pl, h_data, h_par, S) || std::memcmp(h_par, ref.data(), np))
      rc = fail(7, "pipeline encode", c);
    std::memcpy(h_data, erased.data(), nd);
    const xec_status st = xec_pipeline_decode(pl, h_data, h_par, S, bm);
    if (rc == 0 && st != (recoverable ? XEC_SUCCESS : XEC_DECODE_FAILURE)) rc = fail(8, "pipeline status", c);
    if (rc == 0 && std::memcmp(h_data, recoverable ? hd.data() : erased.data(), nd))
      rc = fail(9, "pipeline bytes", c);
    xec_pipeline_destroy(pl);
    delete[] h_data;
    delete[] h_par;
  }
  delete[] bm;
  (void)hipFree(d);
  (void)hipFree(p);
  (void)hipFree(dbm);
  return rc;
}

}  // namespace

int main(int argc, char** argv) {
  const int cases = argc > 1 ? std::atoi(argv[1]) : 60;
  if (xec_init(0) != XEC_SUCCESS) return 2;
  std::mt19937_64 rng(20261016);
  int rc = 0;
  for (int c = 0; c < cases && rc == 0; ++c) rc = one_case(rng, c);
  std::printf(rc == 0 ? "abi_asan ok (%d cases)\n" : "abi_asan FAILED after %d cases\n", cases);
  // leave without the HIP runtime's static teardown (see multi_equiv.cpp)
  std::fflush(stdout);
  std::_Exit(rc == 0 ? 0 : 1);
}
