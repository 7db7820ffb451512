// multi_scatter.cpp -- XorecBenchmarkHipMulti::scatter_from / gather_parity_to
// (GPU test program, built by tests/host/Makefile, run by
// tests/test_plugin_harness.py).
//
// Config 5's exchange in one process: a batch that starts in device 0's HBM
// is scattered over the shards (peer copies; on a one-GPU box the device list
// repeats device 0, so the copies are device copies), every shard encodes its
// range, the parity is gathered back to device 0 and must equal device 0's own
// encode of the whole batch; each shard's data must equal its range of the
// root batch.  Prints the scatter / gather times (information only) and
// "multi_scatter ok".
//
// `multi_scatter --distinct` runs the cases over the distinct devices
// 0 .. min(count, 8) - 1 instead (real peer copies between
// GPUs), and also requires every remote shard to have reached the root by peer
// access (PeerAccess::kEnabled), not by a runtime-staged copy; it needs two
// or more GPUs and exits 3 with a message on fewer.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "xec.h"
#include "xorec_hip_multi_bm.hpp"

namespace {

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int check(size_t S, size_t k, size_t m, size_t bs, std::vector<int> devices, bool need_peer) {
  BenchmarkConfig c{};
  c.message_size = S * k * bs;
  c.block_size = bs;
  c.ec_params = {k + m, k};
  c.num_lost_blocks = 0;
  c.num_cpu_threads = 4;
  c.gpu_computation = true;
  XecPluginOptions opt;
  opt.seeded = true;
  opt.seed = 11;
  opt.devices = devices;
  XorecBenchmarkHipMulti multi(c, opt);
  if (hipSetDevice(0) != hipSuccess) return 20;
  uint8_t *root = nullptr, *root_par = nullptr, *ref_par = nullptr;
  if (hipMalloc(&root, S * k * bs) != hipSuccess || hipMalloc(&root_par, S * m * bs) != hipSuccess ||
      hipMalloc(&ref_par, S * m * bs) != hipSuccess)
    return 21;
  int rc = 0;
  if (xec_fill_splitmix64(root, S, k * bs, 1896, nullptr) != XEC_SUCCESS ||
      xec_encode(root, ref_par, S, bs, k, m, nullptr) != XEC_SUCCESS ||
      hipMemset(root_par, 0xA5, S * m * bs) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    rc = 22;
  double t_sc = 0, t_ga = 0;
  if (rc == 0) {
    const double t0 = now();
    if (multi.scatter_from(root, 0) != 0) rc = 1;
    t_sc = now() - t0;
  }
  if (rc == 0 && multi.encode() != 0) rc = 2;
  if (rc == 0) {
    const double t0 = now();
    if (multi.gather_parity_to(root_par, 0) != 0) rc = 3;
    t_ga = now() - t0;
  }
  size_t most = 0;  // the largest shard: the read-back buffers' size
  for (size_t i = 0; i < multi.num_shards(); ++i) most = std::max(most, multi.shard_count(i));
  std::vector<uint8_t> a(S * m * bs), b(S * m * bs), hd(S * k * bs), sd(most * k * bs),
      sp(most * m * bs);
  (void)hipSetDevice(0);
  if (rc == 0 && (hipMemcpy(a.data(), root_par, a.size(), hipMemcpyDeviceToHost) != hipSuccess ||
                  hipMemcpy(b.data(), ref_par, b.size(), hipMemcpyDeviceToHost) != hipSuccess ||
                  hipMemcpy(hd.data(), root, hd.size(), hipMemcpyDeviceToHost) != hipSuccess))
    rc = 23;
  if (rc == 0 && a != b) rc = 4;  // gathered parity == root's own encode
  for (size_t i = 0; rc == 0 && i < multi.num_shards(); ++i) {
    const size_t f = multi.shard_first(i), n = multi.shard_count(i);
    if (!multi.read_shard(i, sd.data(), sp.data())) rc = 24;
    else if (std::memcmp(sd.data(), hd.data() + f * k * bs, n * k * bs) != 0) rc = 5;
    else if (need_peer && multi.shard_device(i) != 0 &&
             multi.shard_peer_access(i) != xec_hip::PeerAccess::kEnabled)
      rc = 6;  // a remote shard without peer access: its copies were staged
  }
  (void)hipFree(root);
  (void)hipFree(root_par);
  (void)hipFree(ref_par);
  std::printf("S=%zu k=%zu m=%zu bs=%zu shards=%zu: scatter %.3f ms (%.1f GB/s), gather %.3f ms -> %d\n",
              S, k, m, bs, devices.size(), t_sc * 1e3, S * k * bs / t_sc / 1e9, t_ga * 1e3, rc);
  return rc;
}

}  // namespace

int main(int argc, char** argv) {
  struct Case {
    size_t S, k, m, bs;
    std::vector<int> devices;
  };
  std::vector<Case> cases = {
      {64, 16, 1, 1 << 20, {0, 0, 0, 0}},  // config 3's shape, 16 stripes per range
      {37, 8, 4, 65536, {0, 0, 0}},        // ragged ranges, m > 1
      {2, 4, 2, 4096, {0, 0, 0, 0, 0}},    // empty ranges
      {16, 32, 1, 4096, {0}},              // one shard: the copy is the whole batch
      {288, 16, 1, 1 << 20, {0}},          // one 4.5 GiB copy: offsets and sizes past 2^32
  };
  const bool distinct = argc > 1 && std::strcmp(argv[1], "--distinct") == 0;
  if (distinct) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count < 2) {
      std::printf("multi_scatter --distinct: %d GPU(s) visible, needs 2 or more\n", count);
      return 3;
    }
    std::vector<int> all;
    for (int d = 0; d < count && d < 8; ++d) all.push_back(d);
    const size_t n = all.size();
    cases = {
        {64 * n, 16, 1, 1 << 20, all},      // config 3's shape, 64 stripes per device
        {37, 8, 4, 65536, all},             // ragged ranges, m > 1
        {n - 1, 4, 2, 4096, all},           // one empty range (the last device's)
        {576, 16, 1, 1 << 20, {1, 0}},      // 4.5 GiB peer copies: offsets and sizes past 2^32
        {33, 16, 1, 1 << 20, {all[n - 1], all[0]}},  // root's shard second
    };
  }
  for (const Case& c : cases) {
    const int rc = check(c.S, c.k, c.m, c.bs, c.devices, distinct);
    if (rc != 0) {
      std::printf("multi_scatter FAILED (%d)\n", rc);
      std::fflush(stdout);
      std::_Exit(1);
    }
  }
  std::printf("multi_scatter ok\n");
  // Every plugin object is gone by now.  Leave without running the HIP
  // runtime's static destructors: under AddressSanitizer (bin/asan_*) its
  // teardown trips ASan's device-allocator check (sanitizer_allocator_device.h,
  // "dev_runtime_unloaded_") after main has returned, whatever ran before.
  std::fflush(stdout);
  std::_Exit(0);
}
