// latency.cpp -- per-call latency of the C ABI at small messages (the
// reference's 8 MiB rows, final_results.csv), one process per sync mode:
//   latency <mode 0..3> [k m bs S iters]
// mode: 0 default, 1 spin, 2 yield, 3 blocking sync -- set with
// hipSetDeviceFlags BEFORE any other HIP call (afterwards it is ignored).
// Prints median/p10/p90 microseconds for: an empty kernel + stream sync, one
// whose arguments are ~4 KB (what passing a decode work list by value would
// cost), xec_encode + stream sync, xec_encode + event sync, a captured
// hipGraph holding the encode + graph sync, and xec_decode (one lost data
// block per stripe, pinned host bitmap) + stream sync with the automatic and
// the work-list tiling; and xec_decode of a batch without losses, alone and
// + stream sync.
#include <dlfcn.h>
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "xec.h"

__global__ void empty_kernel() {}

struct BigArgs {
  uint32_t n;
  uint32_t v[1000];
};
__global__ void bigarg_kernel(BigArgs a, uint32_t* out) {
  if (threadIdx.x == 0) out[0] = a.v[a.n % 1000];
}
// kernel arguments of the sizes the decode's work-list capacities ship
// (64 / 256 / 1024 entries: 256 B / 1 KiB / 4 KiB)
template <int N>
struct Args {
  uint32_t v[N];
};
template <int N>
__global__ void args_kernel(Args<N> a, uint32_t* out) {
  if (threadIdx.x == 0) out[0] = a.v[N - 1];
}

// Latency probes (round 6, DESIGN.md §4 *Small messages*): one-wave
// workgroups, one 1 KiB chunk each, like the codec's tiles.  load_probe only
// loads (the store is never taken), store_probe only stores, copy_probe loads
// then stores: timed from their own dispatch they split a small codec
// kernel's time into dispatch, load round trip and store drain.
using u32x4 = __attribute__((ext_vector_type(4))) uint32_t;
__global__ void load_probe(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint32_t key) {
  const u32x4 v = __builtin_nontemporal_load(src + blockIdx.x * 64 + threadIdx.x);
  if (v.x == key && v.y == key + 1) dst[blockIdx.x * 64 + threadIdx.x] = v;
}
__global__ void store_probe(u32x4* __restrict__ dst, uint32_t key) {
  const u32x4 v = {key, blockIdx.x, threadIdx.x, 0u};
  __builtin_nontemporal_store(v, dst + blockIdx.x * 64 + threadIdx.x);
}
__global__ void copy_probe(const u32x4* __restrict__ src, u32x4* __restrict__ dst) {
  const u32x4 v = __builtin_nontemporal_load(src + blockIdx.x * 64 + threadIdx.x);
  __builtin_nontemporal_store(v, dst + blockIdx.x * 64 + threadIdx.x);
}

// xec_set_kernel_events is new in round 6: looked up at run time, so this
// tool still runs against an older libxec_hip.so (LD_LIBRARY_PATH) and then
// skips the dispatch-timed measurements
using SetEvents = xec_status (*)(hipEvent_t, hipEvent_t);
static SetEvents set_events() {
  return reinterpret_cast<SetEvents>(dlsym(RTLD_DEFAULT, "xec_set_kernel_events"));
}

static void report(const char* name, std::vector<double>& us) {
  std::sort(us.begin(), us.end());
  const size_t n = us.size();
  std::printf("%-28s median %8.2f us  p10 %8.2f  p90 %8.2f\n", name, us[n / 2], us[n / 10],
              us[n * 9 / 10]);
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
  const size_t k = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 8;
  const size_t m = argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 4;
  const size_t bs = argc > 4 ? std::strtoull(argv[4], nullptr, 10) : 1024;
  const size_t S = argc > 5 ? std::strtoull(argv[5], nullptr, 10) : (8u << 20) / (k * 1024);
  const int iters = argc > 6 ? std::atoi(argv[6]) : 2000;
  // lost data blocks per stripe, one per parity class (classes 0 .. lost-1)
  const size_t lost = argc > 7 ? std::strtoull(argv[7], nullptr, 10) : 1;
  if (lost < 1 || lost > m) {
    std::fprintf(stderr, "lost per stripe must be 1..m\n");
    return 2;
  }
  static const unsigned flags[] = {hipDeviceScheduleAuto, hipDeviceScheduleSpin,
                                   hipDeviceScheduleYield, hipDeviceScheduleBlockingSync};
  CK(hipSetDeviceFlags(flags[mode & 3]));
  if (xec_init(0) != XEC_SUCCESS) return 1;
  // XEC_LAT_OCC=n: xec_set_occupancy(n) for every codec call of this run
  // (0 automatic, 1..7 waves per SIMD, 8 no cap)
  if (const char* o = std::getenv("XEC_LAT_OCC"); o != nullptr && *o != '\0')
    if (xec_set_occupancy(std::atoi(o)) != XEC_SUCCESS) return 1;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void *d, *p;
  CK(hipMalloc(&d, S * k * bs));
  CK(hipMalloc(&p, S * m * bs));
  CK(hipMemset(d, 0x5a, S * k * bs));
  CK(hipDeviceSynchronize());
  std::printf("mode %d  k=%zu m=%zu bs=%zu S=%zu (%zu KiB data)\n", mode, k, m, bs, S,
              S * k * bs >> 10);
  using clk = std::chrono::steady_clock;
  auto us_since = [](clk::time_point t0) {
    return std::chrono::duration<double, std::micro>(clk::now() - t0).count();
  };
  std::vector<double> t;
  for (int i = 0; i < iters + 50; ++i) {
    auto t0 = clk::now();
    empty_kernel<<<1, 64, 0, s>>>();
    CK(hipStreamSynchronize(s));
    if (i >= 50) t.push_back(us_since(t0));
  }
  report("empty kernel + stream sync", t);
  t.clear();
  for (int i = 0; i < iters + 50; ++i) {
    auto t0 = clk::now();
    empty_kernel<<<1, 64, 0, s>>>();
    const double us = us_since(t0);
    CK(hipStreamSynchronize(s));
    if (i >= 50) t.push_back(us);
  }
  report("empty kernel, call only", t);
  t.clear();
  // the copy probe over the batch's 1 KiB tiles (the encode's grid at m = 1),
  // launched with <<<>>>, without and with an LDS reservation of L bytes
  // (XEC_LAT_LDS, default 10240: the residency cap's reservation at 8 members)
  {
    const uint32_t tiles = (uint32_t)std::min<size_t>(S * m * bs / 1024, S * k * bs / 1024);
    const char* le = std::getenv("XEC_LAT_LDS");
    const uint32_t lds = le != nullptr && *le != '\0' ? (uint32_t)std::atoi(le) : 10240u;
    for (uint32_t l : {0u, lds}) {
      for (int i = 0; i < iters + 50; ++i) {
        auto t0 = clk::now();
        hipLaunchKernelGGL(copy_probe, dim3(tiles), dim3(64), l, s,
                           static_cast<const u32x4*>(d), static_cast<u32x4*>(p));
        CK(hipStreamSynchronize(s));
        if (i >= 50) t.push_back(us_since(t0));
      }
      char nm[64];
      std::snprintf(nm, sizeof nm, "copy x%u lds %u + sync", tiles, l);
      report(nm, t);
      t.clear();
    }
    for (int i = 0; i < iters + 50; ++i) {
      auto t0 = clk::now();
      hipLaunchKernelGGL(copy_probe, dim3(tiles), dim3(64), 0, s, static_cast<const u32x4*>(d),
                         static_cast<u32x4*>(p));
      const double us = us_since(t0);
      CK(hipStreamSynchronize(s));
      if (i >= 50) t.push_back(us);
    }
    report("copy, call only", t);
    t.clear();
  }
  {
    static BigArgs ba;
    ba.n = 7;
    for (int i = 0; i < 1000; ++i) ba.v[i] = i;
    uint32_t* dout;
    CK(hipMalloc(&dout, 4));
    for (int i = 0; i < iters + 50; ++i) {
      auto t0 = clk::now();
      ba.n = i;
      bigarg_kernel<<<1, 64, 0, s>>>(ba, dout);
      CK(hipStreamSynchronize(s));
      if (i >= 50) t.push_back(us_since(t0));
    }
    uint32_t hv = 0;
    CK(hipMemcpy(&hv, dout, 4, hipMemcpyDeviceToHost));
    if (hv != (uint32_t)((iters + 49) % 1000)) {
      std::fprintf(stderr, "bigarg kernel read %u\n", hv);
      return 3;
    }
    report("4 KB-arg kernel + stream sync", t);
    t.clear();
    auto sized = [&](auto tag, const char* name) -> int {
      constexpr int N = decltype(tag)::value;
      static Args<N> a;
      for (int i = 0; i < iters + 50; ++i) {
        auto t0 = clk::now();
        a.v[N - 1] = i;
        args_kernel<N><<<1, 64, 0, s>>>(a, dout);
        CK(hipStreamSynchronize(s));
        if (i >= 50) t.push_back(us_since(t0));
      }
      report(name, t);
      t.clear();
      return 0;
    };
    if (sized(std::integral_constant<int, 64>{}, "256 B-arg kernel + sync") ||
        sized(std::integral_constant<int, 256>{}, "1 KB-arg kernel + sync") ||
        sized(std::integral_constant<int, 1024>{}, "4 KB-arg kernel (tmpl) + sync"))
      return 1;
  }
  for (int i = 0; i < iters + 50; ++i) {
    auto t0 = clk::now();
    if (xec_encode(d, p, S, bs, k, m, s) != XEC_SUCCESS) return 2;
    CK(hipStreamSynchronize(s));
    if (i >= 50) t.push_back(us_since(t0));
  }
  report("xec_encode + stream sync", t);
  t.clear();
  for (int i = 0; i < iters + 50; ++i) {
    auto t0 = clk::now();
    if (xec_encode(d, p, S, bs, k, m, s) != XEC_SUCCESS) return 2;
    const double us = us_since(t0);
    CK(hipStreamSynchronize(s));
    if (i >= 50) t.push_back(us);
  }
  report("xec_encode, call only", t);
  t.clear();
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (int i = 0; i < iters + 50; ++i) {
    auto t0 = clk::now();
    if (xec_encode(d, p, S, bs, k, m, s) != XEC_SUCCESS) return 2;
    CK(hipEventRecord(ev, s));
    CK(hipEventSynchronize(ev));
    if (i >= 50) t.push_back(us_since(t0));
  }
  report("xec_encode + event sync", t);
  t.clear();
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  if (xec_encode(d, p, S, bs, k, m, s) != XEC_SUCCESS) return 2;
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < iters + 50; ++i) {
    auto t0 = clk::now();
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    if (i >= 50) t.push_back(us_since(t0));
  }
  report("graph(encode) + stream sync", t);
  t.clear();
  // device time of the encode alone
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 200; ++i) {
    CK(hipEventRecord(e0, s));
    if (xec_encode(d, p, S, bs, k, m, s) != XEC_SUCCESS) return 2;
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms * 1e3);
  }
  report("encode device time (events)", t);
  t.clear();
  // the encode kernel alone: events recorded by its own dispatch
  const SetEvents arm = set_events();
  for (int i = 0; arm != nullptr && i < 500; ++i) {
    if (arm(e0, e1) != XEC_SUCCESS) return 2;
    if (xec_encode(d, p, S, bs, k, m, s) != XEC_SUCCESS) return 2;
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms * 1e3);
  }
  if (arm != nullptr) report("encode kernel (dispatch)", t);
  t.clear();
  // the probes, timed the same way (hipExtLaunchKernelGGL records e0 / e1 at
  // the kernel's own dispatch); grids of 1 and of the batch's 1 KiB tiles
  {
    const uint32_t tiles = (uint32_t)std::min<size_t>(S * m * bs / 1024, S * k * bs / 1024);
    const u32x4* src = static_cast<const u32x4*>(d);
    u32x4* dst = static_cast<u32x4*>(p);
    auto timed = [&](const char* name, auto launch) -> int {
      for (int i = 0; i < 500; ++i) {
        launch();
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms * 1e3);
      }
      report(name, t);
      t.clear();
      return 0;
    };
    char nm[64];
    for (uint32_t grid : {1u, tiles}) {
      std::snprintf(nm, sizeof nm, "empty x%u (dispatch)", grid);
      if (timed(nm, [&] { hipExtLaunchKernelGGL(empty_kernel, dim3(grid), dim3(64), 0, s, e0, e1, 0); }))
        return 1;
      std::snprintf(nm, sizeof nm, "load x%u (dispatch)", grid);
      if (timed(nm, [&] { hipExtLaunchKernelGGL(load_probe, dim3(grid), dim3(64), 0, s, e0, e1, 0, src, dst, 0x12345u); }))
        return 1;
      std::snprintf(nm, sizeof nm, "store x%u (dispatch)", grid);
      if (timed(nm, [&] { hipExtLaunchKernelGGL(store_probe, dim3(grid), dim3(64), 0, s, e0, e1, 0, dst, 7u); }))
        return 1;
      std::snprintf(nm, sizeof nm, "copy x%u (dispatch)", grid);
      if (timed(nm, [&] { hipExtLaunchKernelGGL(copy_probe, dim3(grid), dim3(64), 0, s, e0, e1, 0, src, dst); }))
        return 1;
    }
  }
  // decode: `lost` data blocks per stripe; with one, (7c) mod k (bench.py's
  // pattern), with more, block j + m * ((7c) mod (k/m)) of classes j < lost
  uint8_t* h_bm;
  uint8_t* d_bm;
  CK(hipHostMalloc(reinterpret_cast<void**>(&h_bm), S * (k + m), hipHostMallocDefault));
  CK(hipMalloc(reinterpret_cast<void**>(&d_bm), S * (k + m)));
  for (size_t c = 0; c < S; ++c) {
    for (size_t i = 0; i < k + m; ++i) h_bm[c * (k + m) + i] = 1;
    if (lost == 1) {
      h_bm[c * (k + m) + (7 * c) % k] = 0;
    } else {
      for (size_t j = 0; j < lost; ++j) h_bm[c * (k + m) + j + m * ((7 * c) % (k / m))] = 0;
    }
  }
  std::printf("decode: %zu lost data block(s) per stripe, %zu in all\n", lost, lost * S);
  for (int tiling : {0, 3}) {
    if (xec_set_decode_tiling(tiling) != XEC_SUCCESS) return 2;
    for (int i = 0; i < iters + 50; ++i) {
      auto t0 = clk::now();
      if (xec_decode(d, p, S, bs, k, m, h_bm, d_bm, s) != XEC_SUCCESS) return 2;
      CK(hipStreamSynchronize(s));
      if (i >= 50) t.push_back(us_since(t0));
    }
    report(tiling ? "xec_decode list + sync" : "xec_decode auto + sync", t);
    t.clear();
  }
  xec_set_decode_tiling(0);
  for (int i = 0; arm != nullptr && i < 500; ++i) {
    if (arm(e0, e1) != XEC_SUCCESS) return 2;
    if (xec_decode(d, p, S, bs, k, m, h_bm, d_bm, s) != XEC_SUCCESS) return 2;
    CK(hipStreamSynchronize(s));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms * 1e3);
  }
  if (arm != nullptr) report("decode kernel (dispatch)", t);
  t.clear();
  // the host time of the decode call alone (its stream synchronised outside
  // the timed region): what a caller that does not wait pays per call
  for (int i = 0; i < iters + 50; ++i) {
    auto t0 = clk::now();
    if (xec_decode(d, p, S, bs, k, m, h_bm, d_bm, s) != XEC_SUCCESS) return 2;
    const double us = us_since(t0);
    CK(hipStreamSynchronize(s));
    if (i >= 50) t.push_back(us);
  }
  report("xec_decode auto, call only", t);
  t.clear();
  // decode of a batch without losses (the reference's lost=0 rows): the host
  // scan finds nothing, so nothing is queued; alone and + stream sync
  for (size_t i = 0; i < S * (k + m); ++i) h_bm[i] = 1;
  for (int sync : {0, 1}) {
    for (int i = 0; i < iters + 50; ++i) {
      auto t0 = clk::now();
      if (xec_decode(d, p, S, bs, k, m, h_bm, d_bm, s) != XEC_SUCCESS) return 2;
      if (sync) CK(hipStreamSynchronize(s));
      if (i >= 50) t.push_back(us_since(t0));
    }
    report(sync ? "xec_decode no loss + sync" : "xec_decode no loss", t);
    t.clear();
  }
  return 0;
}
