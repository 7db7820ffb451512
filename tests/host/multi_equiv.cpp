// multi_equiv.cpp -- XorecBenchmarkHipMulti against XorecBenchmarkHip (GPU test
// program, built by tests/host/Makefile, run by tests/test_plugin_harness.py).
//
// The multi-device plugin over a device list that repeats device 0 (several
// stripe ranges on one GPU, each with its own stream and buffers) must give
// the same bytes as the one-device plugin for the same config and seed: after
// setup + encode (data and parity), after simulate_data_loss (the erased
// batch) and after decode (the rebuilt data), and both must pass
// check_for_corruption.  Prints "multi_equiv ok" and exits 0 on success.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "xorec_hip_bm.hpp"
#include "xorec_hip_multi_bm.hpp"

namespace {

// Makes stripe c unrecoverable on the host bitmap: its first lost data block's
// class also loses its parity (is_recoverable, xorec_utils.hpp:160-175).
void spoil(uint8_t* bm, size_t c, size_t k, size_t m) {
  uint8_t* row = bm + c * (k + m);
  for (size_t i = 0; i < k; ++i)
    if (!row[i]) {
      row[k + i % m] = 0;
      return;
    }
}

class Multi : public XorecBenchmarkHipMulti {
 public:
  using XorecBenchmarkHipMulti::XorecBenchmarkHipMulti;
  void spoil_stripe(size_t c) { spoil(m_block_bitmap.get(), c, m_chunk_data_blocks, m_chunk_parity_blocks); }
};

class Single : public XorecBenchmarkHip {
 public:
  using XorecBenchmarkHip::XorecBenchmarkHip;
  void spoil_stripe(size_t c) { spoil(m_block_bitmap.get(), c, m_chunk_data_blocks, m_chunk_parity_blocks); }
  void read(std::vector<uint8_t>& d, std::vector<uint8_t>& p) const {
    d.resize(m_chunks * m_chunk_data_size);
    p.resize(m_chunks * m_chunk_parity_size);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(d.data(), m_data_buf.get(), d.size(), hipMemcpyDeviceToHost);
    (void)hipMemcpy(p.data(), m_parity_buf.get(), p.size(), hipMemcpyDeviceToHost);
  }
};

void read_multi(const XorecBenchmarkHipMulti& b, size_t kbs, size_t mbs,
                std::vector<uint8_t>& d, std::vector<uint8_t>& p, size_t S) {
  d.assign(S * kbs, 0);
  p.assign(S * mbs, 0);
  for (size_t i = 0; i < b.num_shards(); ++i)
    if (!b.read_shard(i, d.data() + b.shard_first(i) * kbs, p.data() + b.shard_first(i) * mbs))
      std::fprintf(stderr, "read_shard %zu failed\n", i);
}

int check(size_t S, size_t k, size_t m, size_t bs, size_t lost, std::vector<int> devices,
          bool unrecoverable = false) {
  BenchmarkConfig c{};
  c.message_size = S * k * bs;
  c.block_size = bs;
  c.ec_params = {k + m, k};
  c.num_lost_blocks = lost;
  c.num_cpu_threads = 4;
  c.gpu_computation = true;
  XecPluginOptions opt;
  opt.seeded = true;
  opt.seed = 5;
  opt.devices = devices;
  Single one(c, opt);
  Multi multi(c, opt);
  if (multi.num_shards() != devices.size()) return 10;
  std::vector<uint8_t> d1, p1, dn, pn;
  int step = 0;
  auto same = [&](bool parity) {
    ++step;
    one.read(d1, p1);
    read_multi(multi, k * bs, m * bs, dn, pn, S);
    if (d1 != dn) return false;
    return !parity || p1 == pn;
  };
  one.setup();
  multi.setup();
  if (one.encode() != 0 || multi.encode() != 0) return 1;
  if (!same(true)) return 2;
  one.simulate_data_loss();
  multi.simulate_data_loss();
  if (!same(true)) return 3;
  if (lost > 0 && one.check_for_corruption()) return 4;  // the erasure must show
  if (unrecoverable) {
    // the LAST stripe (last shard) cannot be rebuilt: both plugins fail the
    // whole batch and touch nothing, on one device or on several
    one.spoil_stripe(S - 1);
    multi.spoil_stripe(S - 1);
    if (one.decode() == 0 || multi.decode() == 0) return 8;
    if (!same(true)) return 9;
    return 0;
  }
  if (one.decode() != 0 || multi.decode() != 0) return 5;
  if (!same(false)) return 6;
  if (!one.check_for_corruption() || !multi.check_for_corruption()) return 7;
  return 0;
}

}  // namespace

int main() {
  struct Case {
    size_t S, k, m, bs, lost;
    std::vector<int> devices;
    bool unrecoverable = false;
  } cases[] = {
      {13, 8, 4, 4096, 3, {0, 0, 0}},      // uneven ranges: 5, 4, 4 stripes
      {7, 16, 1, 65536, 1, {0, 0}},        // 4 + 3
      {2, 32, 8, 1024, 8, {0, 0, 0, 0}},   // more shards than stripes: two empty
      {64, 16, 4, 8192, 0, {0}},           // one shard, nothing lost
      {13, 8, 4, 4096, 2, {0, 0, 0}, true},  // last stripe unrecoverable: nothing rebuilt anywhere
      {9, 16, 1, 8192, 1, {0, 0}, true},
  };
  for (const Case& x : cases) {
    const int rc = check(x.S, x.k, x.m, x.bs, x.lost, x.devices, x.unrecoverable);
    if (rc != 0) {
      std::printf("multi_equiv FAILED at S=%zu k=%zu m=%zu bs=%zu lost=%zu shards=%zu: %d\n", x.S,
                  x.k, x.m, x.bs, x.lost, x.devices.size(), rc);
      std::fflush(stdout);
      std::_Exit(1);
    }
  }
  std::printf("multi_equiv ok\n");
  // Every plugin object is gone by now.  Leave without running the HIP
  // runtime's static destructors: under AddressSanitizer (bin/asan_*) its
  // teardown trips ASan's device-allocator check (sanitizer_allocator_device.h,
  // "dev_runtime_unloaded_") after main has returned, whatever ran before.
  std::fflush(stdout);
  std::_Exit(0);
}
