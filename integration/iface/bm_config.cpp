// bm_config.cpp -- the reference's sweep vectors (src/benchmark/bm_config.cpp:3-23)
// from which its get_gpu_configs (src/utils/benchmark_suite.cpp:252-277) forms
// the GPU cross product; and get_version_name (src/xorec/xorec_utils.cpp:4-16).
#include "bm_config.hpp"

#include "utils.hpp"

const std::vector<size_t> VAR_BLOCK_SIZES = {1 KiB, 2 KiB, 4 KiB, 8 KiB};
const std::vector<ECTuple> VAR_EC_PARAMS = {
    {8 + 4, 8}, {16 + 4, 16}, {16 + 8, 16}, {32 + 4, 32}, {32 + 8, 32}};
const std::vector<size_t> VAR_NUM_CPU_THREADS = {1, 2, 4, 8, 16, 32};
const std::vector<size_t> VAR_NUM_LOST_BLOCKS = {0, 1, 2, 4, 8};
const std::vector<size_t> VAR_NUM_GPU_BLOCKS = {256};
const std::vector<size_t> VAR_NUM_THREADS_PER_BLOCK = {512};

std::string get_version_name(XorecVersion version) {
  switch (version) {
    case XorecVersion::Scalar: return "Scalar";
    case XorecVersion::SSE2: return "SSE2";
    case XorecVersion::AVX2: return "AVX2";
    case XorecVersion::AVX512: return "AVX-512";
  }
  throw_error("Invalid XorecVersion");
}
