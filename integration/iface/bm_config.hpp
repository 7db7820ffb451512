// bm_config.hpp -- this repository's restatement of the reference's per-run
// configuration header (src/benchmark/bm_config.hpp:1-57), for builds where the
// reference is not mounted.  What a plugin sees of it:
//   * BenchmarkConfig -- the fields of bm_config.hpp:25-43, same names, types,
//     order and defaults (plugin constructors take one);
//   * the KiB / MiB literal suffix macros, ECTuple = (total blocks, data
//     blocks), MESSAGE_SIZE and the sweep vectors (defined in bm_config.cpp);
//   * BenchmarkFunction, whose benchmark::State parameter (Google Benchmark)
//     and the ConsoleReporter pointer are only named, never used: both are
//     declared as incomplete types here.
#ifndef BM_CONFIG_HPP
#define BM_CONFIG_HPP

#include <cstddef>
#include <cstdint>
#include <tuple>
#include <vector>

#include "xorec_utils.hpp"

#define KiB *1024
#define MiB *1024*1024

class ConsoleReporter;
namespace benchmark {
class State;
}

using ECTuple = std::tuple<size_t, size_t>;

struct BenchmarkConfig {
  // the batch: message bytes, block bytes, (k + m, k), losses per stripe
  size_t message_size;
  size_t block_size;
  ECTuple ec_params;
  size_t num_lost_blocks;
  // host threads of the CPU codecs
  size_t num_cpu_threads;
  // timed and untimed iterations of BM_generic
  int num_iterations;
  int num_warmup_iterations;
  XorecVersion xorec_version = XorecVersion::Scalar;
  // GPU codecs; the grid of the reference's CUDA kernels
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
