// xec_plugin_options.hpp -- what the MI355X plugins take beyond the reference's
// BenchmarkConfig (which they use as it is: bm_config.hpp:25-43).  The
// reference registers a plugin with its one-argument constructor
// (INTEGRATION.md §3), which means the defaults below: the reference's own
// behaviour -- device 0, wall-clock payloads and erasure draws from its
// utils.hpp.  This repository's harness (bin/xec_bench, bin/xec_multi_leg)
// passes options for reproducible runs and device lists.
#ifndef XEC_PLUGIN_OPTIONS_HPP
#define XEC_PLUGIN_OPTIONS_HPP

#include <cstdint>
#include <vector>

struct XecPluginOptions {
  // XorecBenchmarkHip's device (the reference's GPU plugin is pinned to
  // device 0, xorec_gpu_cmp.cu:7-16).
  int device = 0;
  // XorecBenchmarkHipMulti's devices, one stripe range each, repeats allowed;
  // empty = the XEC_DEVICES environment variable, else every visible device.
  std::vector<int> devices;
  // false: payloads from the reference's write_validation_pattern on the host
  // (one upload per setup) and erasures from its select_lost_blocks, both
  // seeded by the wall clock.  true: payloads written on the device
  // (xec_write_validation_pattern) and erasures drawn on the host
  // (xec_select_lost_blocks), both from `seed`, a fresh round per setup().
  bool seeded = false;
  uint64_t seed = 0;
  // check_for_corruption on the host after copying the data back, as the
  // reference (xorec_gpu_cmp_bm.cpp:91-104); false = on the device
  // (xec_validate_blocks), which checks the same checksum.
  bool host_check = false;
  // hipSetDeviceFlags before the first allocation: 0 leave the runtime
  // default, 1 spin, 2 yield, 3 blocking sync.
  int sync_mode = 0;
};

#endif  // XEC_PLUGIN_OPTIONS_HPP
