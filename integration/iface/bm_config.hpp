// bm_config.hpp -- this repository's restatement of the reference's
// src/benchmark/bm_config.hpp:1-57: the per-run BenchmarkConfig every plugin
// constructor takes, the KiB / MiB literal macros and the sweep vectors
// (defined in bm_config.cpp, as the reference's src/benchmark/bm_config.cpp:3-23).
//
// The reference pulls ConsoleReporter and benchmark::State in through Google
// Benchmark (console_reporter.hpp); the config only names them as incomplete
// types, so they are declared here and nothing else of Google Benchmark is
// needed.
#ifndef BM_CONFIG_HPP
#define BM_CONFIG_HPP

#define KiB *1024
#define MiB *1024*1024

#include <cstddef>
#include <cstdint>
#include <tuple>
#include <vector>

#include "xorec_utils.hpp"

namespace benchmark {
class State;
}
class ConsoleReporter;

// (total blocks, data blocks) of one stripe, bm_config.hpp:18
using ECTuple = std::tuple<size_t, size_t>;

// bm_config.hpp:25-43, field for field
struct BenchmarkConfig {
  size_t message_size;     // bytes of data per batch (all stripes)
  size_t block_size;       // bytes per block
  ECTuple ec_params;       // (k + m, k)
  size_t num_lost_blocks;  // blocks lost per stripe (data or parity)

  size_t num_cpu_threads;

  int num_iterations;
  int num_warmup_iterations;

  XorecVersion xorec_version = XorecVersion::Scalar;

  bool gpu_computation;
  size_t num_gpu_blocks = 0;
  size_t threads_per_gpu_block = 0;

  ConsoleReporter* reporter = nullptr;
};

using BenchmarkFunction = void (*)(benchmark::State&, const BenchmarkConfig&);

constexpr size_t MESSAGE_SIZE = 8 MiB;
extern const std::vector<size_t> VAR_BLOCK_SIZES;
extern const std::vector<ECTuple> VAR_EC_PARAMS;
extern const std::vector<size_t> VAR_NUM_CPU_THREADS;
extern const std::vector<size_t> VAR_NUM_LOST_BLOCKS;
extern const std::vector<size_t> VAR_NUM_GPU_BLOCKS;
extern const std::vector<size_t> VAR_NUM_THREADS_PER_BLOCK;

#endif  // BM_CONFIG_HPP
