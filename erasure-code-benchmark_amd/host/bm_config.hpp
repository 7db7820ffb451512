// bm_config.hpp -- benchmark configuration for the XOR-EC HIP plugin.
//
// Mirrors the fields and meaning of the reference's BenchmarkConfig
// (src/benchmark/bm_config.hpp:25-43) so a config built for the reference's
// "xorec-gpu" plugin means the same thing here.  Fields that only exist for
// the reference's CUDA launch (num_gpu_blocks / threads_per_gpu_block) are kept
// for the CSV schema; the HIP path chooses its own launch shape.
#pragma once

#include <cstddef>
#include <cstdint>
#include <tuple>
#include <vector>

namespace xec {

using ECTuple = std::tuple<size_t, size_t>;  // (total blocks, data blocks), bm_config.hpp:18

struct BenchmarkConfig {
  size_t message_size = 0;      // bytes of data per batch (all stripes)
  size_t block_size = 0;        // bytes per block (shard)
  ECTuple ec_params{0, 0};      // (k + m, k)
  size_t num_lost_blocks = 0;   // lost blocks per stripe (data or parity)
  size_t num_cpu_threads = 1;   // host threads for setup / validation
  int num_iterations = 10;      // timed iterations (benchmark_suite.cpp:30)
  int num_warmup_iterations = 0;
  bool gpu_computation = true;
  size_t num_gpu_blocks = 0;          // CSV only (reference launch grid)
  size_t threads_per_gpu_block = 256; // CSV only
  int device_id = 0;            // new: HIP device of this process
  uint64_t seed = 0;            // new: explicit seed (reference seeds from the clock)
  bool host_validation = false; // new: true = payload written/checked on the host and copied
                                //   (the reference's way, xorec_gpu_cmp_bm.cpp:25-37,91-104);
                                //   false = on the device (xec_write_validation_pattern)
  int sync_mode = 0;            // new: 0 runtime default, 1 spin, 2 yield, 3 blocking sync
                                // (hipSetDeviceFlags; CUDA's default "auto" spins when
                                // contexts < cores, which is what the reference ran under)
  std::vector<int> devices;     // new: XorecBenchmarkHipMulti's devices, one stripe range
                                // each (repeats allowed); empty = every visible device
};

// The reference's sweep vectors (src/benchmark/bm_config.cpp:3-23,
// bm_config.hpp:51) from which get_gpu_configs (benchmark_suite.cpp:252-277)
// forms the GPU cross product.
constexpr size_t kMessageSize = 8u << 20;  // MESSAGE_SIZE = 8 MiB
inline const std::vector<size_t> kVarBlockSizes = {1u << 10, 2u << 10, 4u << 10, 8u << 10};
inline const std::vector<ECTuple> kVarEcParams = {
    {4 + 8, 8}, {4 + 16, 16}, {8 + 16, 16}, {4 + 32, 32}, {8 + 32, 32}};
inline const std::vector<size_t> kVarNumLostBlocks = {0, 1, 2, 4, 8};
inline const std::vector<size_t> kVarNumGpuBlocks = {256};
inline const std::vector<size_t> kVarNumThreadsPerBlock = {512};

inline size_t data_blocks(const BenchmarkConfig& c) { return std::get<1>(c.ec_params); }
inline size_t parity_blocks(const BenchmarkConfig& c) {
  return std::get<0>(c.ec_params) - std::get<1>(c.ec_params);
}

}  // namespace xec
