// tsan_overrides.cpp -- per-thread tuning overrides under ThreadSanitizer on the
// GPU box (built by tests/host/Makefile as bin/tsan_overrides: csrc/xec_api.cpp,
// xec_scan.cpp and xec_pipeline.cpp compiled in with host-only TSan, the
// kernels as usual; run by tests/test_plugin_harness.py).
//
// Two threads, each on its own stream and buffers, set DIFFERENT overrides
// (xec_set_launch, xec_set_occupancy, xec_set_decode_tiling,
// xec_set_validate_kernel) and then run encode -> erase -> decode -> validate
// many times, interleaved with each other.  Checked every iteration:
//   - the decode tiling this thread's call launched (xec_decode_tiling_used) is
//     the one THIS thread forced, never the other thread's;
//   - parity equals a host XOR of each class; the decode restores the data;
//   - a third thread that set nothing gets the automatic choice.
// Any data race on the override state is a TSan report (non-zero exit).
// Prints "tsan_overrides ok".
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "xec.h"

namespace {

std::atomic<int> g_failures{0};

void fail(int t, int it, const char* what) {
  std::printf("thread %d iteration %d: %s\n", t, it, what);
  g_failures.fetch_add(1);
}

// k=8+2, 4 KiB blocks: every stripe loses one data block in each class (so
// class tiles are a valid forced choice; the automatic choice for this dense
// multi-erasure batch of 96 stripes is class tiles over kernel-argument loss
// masks -- three threads, three different tilings).
constexpr size_t kK = 8, kM = 2, kBs = 4096, kS = 96, kRow = kK + kM;

void worker(int t, int tiling, int unroll, int threads, int occupancy, int validate_mode,
            int iterations) {
  if (tiling >= 0 && xec_set_decode_tiling(tiling) != XEC_SUCCESS) return fail(t, -1, "set tiling");
  if (unroll >= 0 && xec_set_launch(unroll, 0, 0, threads) != XEC_SUCCESS)
    return fail(t, -1, "set launch");
  if (occupancy >= 0 && xec_set_occupancy(occupancy) != XEC_SUCCESS)
    return fail(t, -1, "set occupancy");
  if (validate_mode >= 0 && xec_set_validate_kernel(validate_mode) != XEC_SUCCESS)
    return fail(t, -1, "set validate");
  hipStream_t s = nullptr;
  uint8_t *d = nullptr, *p = nullptr, *dbm = nullptr, *hbm = nullptr;
  const size_t nd = kS * kK * kBs, np = kS * kM * kBs;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) || hipMalloc(&d, nd) ||
      hipMalloc(&p, np) || hipMalloc(&dbm, kS * kRow) || hipHostMalloc(&hbm, kS * kRow, 0))
    return fail(t, -1, "alloc");
  std::vector<uint8_t> orig(nd), got(nd), hp(np), ref(np);
  for (size_t c = 0; c < kS; ++c) {  // per stripe: lose one member of each class
    std::memset(hbm + c * kRow, 1, kRow);
    for (size_t j = 0; j < kM; ++j) hbm[c * kRow + j + kM * ((c + j + t) % (kK / kM))] = 0;
  }
  // auto: dense multi-erasure over 96 stripes -> the kernel-argument masks
  const int want = tiling > 0 ? tiling : XEC_TILING_ARG_MASK;
  for (int it = 0; it < iterations; ++it) {
    if (xec_fill_splitmix64(d, kS, kK * kBs, 1000 * t + it, s) ||
        xec_encode(d, p, kS, kBs, kK, kM, s) ||
        hipMemcpyAsync(orig.data(), d, nd, hipMemcpyDeviceToHost, s) ||
        hipMemcpyAsync(hp.data(), p, np, hipMemcpyDeviceToHost, s) || hipStreamSynchronize(s))
      return fail(t, it, "encode");
    std::fill(ref.begin(), ref.end(), 0);
    for (size_t c = 0; c < kS; ++c)
      for (size_t i = 0; i < kK; ++i)
        for (size_t b = 0; b < kBs; ++b) ref[(c * kM + i % kM) * kBs + b] ^= orig[(c * kK + i) * kBs + b];
    if (hp != ref) return fail(t, it, "parity");
    if (hipMemcpyAsync(dbm, hbm, kS * kRow, hipMemcpyHostToDevice, s) ||
        xec_erase(d, p, kS, kBs, kK, kM, dbm, s) ||
        xec_decode(d, p, kS, kBs, kK, kM, hbm, dbm, s))
      return fail(t, it, "erase/decode");
    if (xec_decode_tiling_used() != want) return fail(t, it, "another thread's tiling");
    if (hipMemcpyAsync(got.data(), d, nd, hipMemcpyDeviceToHost, s) || hipStreamSynchronize(s))
      return fail(t, it, "copy");
    if (got != orig) return fail(t, it, "decoded data");
    // the validation kernels under this thread's xec_set_validate_kernel
    uint32_t* d_bad = reinterpret_cast<uint32_t*>(dbm);
    uint32_t bad = 1;
    if (xec_write_validation_pattern(d, kS * kK, kBs, it, s) ||
        xec_validate_blocks(d, kS * kK, kBs, d_bad, s) ||
        hipMemcpyAsync(&bad, d_bad, sizeof bad, hipMemcpyDeviceToHost, s) || hipStreamSynchronize(s))
      return fail(t, it, "validate");
    if (bad != 0) return fail(t, it, "validation pattern");
  }
  (void)hipStreamDestroy(s);
  (void)hipFree(d);
  (void)hipFree(p);
  (void)hipFree(dbm);
  (void)hipHostFree(hbm);
}

}  // namespace

int main() {
  if (xec_init(0) != XEC_SUCCESS) {
    std::printf("xec_init failed\n");
    return 2;
  }
  const int iters = 40;
  // thread 0: stripe tiles, two granules per lane, 256-thread workgroups, no cap
  // thread 1: class tiles, defaults otherwise, one wave per SIMD, lane validation
  // thread 2: sets nothing (automatic everything)
  std::thread a(worker, 0, XEC_TILING_STRIPE, 2, 256, 8, 2, iters);
  std::thread b(worker, 1, XEC_TILING_CLASS, 1, 64, 1, 1, iters);
  std::thread c(worker, 2, -1, -1, 0, -1, -1, iters);
  a.join();
  b.join();
  c.join();
  // the main thread set nothing either: its next decode is automatic too
  if (g_failures.load() != 0) return 1;
  std::printf("tsan_overrides ok\n");
  return 0;
}
