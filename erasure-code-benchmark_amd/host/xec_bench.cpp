// xec_bench.cpp -- command-line harness with the reference's CLI contract
// (src/utils/benchmark_suite.cpp:102-212) for the HIP XOR-EC plugins,
// registered as GPU algorithms "xorec-hip" (one device, XorecBenchmarkHip) and
// "xorec-hip-multi" (the batch's stripes split over several devices of this
// process, XorecBenchmarkHipMulti) beside the reference's "xorec-gpu"
// (benchmark_suite.cpp:56-62; runners.cpp:43-45).
//
//   xec_bench -g xorec-hip[,xorec-hip-multi] [-f out.csv] [-a] [-i iters] [-w warmup]
//             [-s simd,...] [-h]
//
//   -f, --file        output CSV (must contain ".csv"; default results.csv); a bare
//                     file name lands in the raw-results directory, ../results/raw/
//                     by default as in the reference (RAW_DIR + OUTPUT_FILE,
//                     benchmark_suite.cpp:27,346, where scripts/utils/data.py
//                     reads it); a path with a '/' is used as given
//   -a, --append      append rows without a header (default: overwrite + header,
//                     csv_reporter.cpp:11-19)
//   -i, --iterations  timed iterations per config (> 0, default 10)
//   -w, --warmup      warm-up iterations per config (>= 0, default 0)
//   -g, --gpu         GPU algorithms, comma separated: xorec-hip, xorec-hip-multi
//   -c, --cpu         CPU algorithms are outside this build (error)
//   -s, --simd        CPU XOR-EC SIMD versions (scalar, sse2, avx2, avx512): validated
//                     like the reference; they select CPU variants only, so no effect here
// With -g and no config options, the configs are the reference's GPU cross
// product (get_gpu_configs, benchmark_suite.cpp:252-277, over the vectors of
// bm_config.cpp:3-23): 8 MiB messages x block sizes x EC params x lost blocks
// (<= m) x 256 GPU blocks x 512 threads, one 20-column CSV row each, in the
// reference's order, algorithm by algorithm (get_benchmarks, :279-311).
//
// Extensions (long options only):
//   --message B --block B --data K --parity M --lost L   one config instead of the sweep
//                                    (sizes accept K/M/G suffixes, binary)
//   --sweep FILE     configs from FILE, one "message block k m lost" per line
//   --threads N      host threads for host-side validation (default: all)
//   --device D       HIP device of xorec-hip (default 0)
//   --devices LIST   devices of xorec-hip-multi, comma separated, repeats allowed
//                    (default: every visible device)
//   --seed S         seed of payloads (written on the device) and erasure draws
//                    (default 0; XecPluginOptions::seeded)
//   --sync MODE      hipSetDeviceFlags: 0 default, 1 spin, 2 yield, 3 blocking
//   --host-validation  the reference's own way: payloads from its wall-clock
//                    write_validation_pattern on the host + one copy, erasures from
//                    its select_lost_blocks, the check on the host after a copy back
//                    (--seed is then unused)
// The plugins are integration/xorec_hip_bm.cpp / xorec_hip_multi_bm.cpp -- the
// drop-in sources themselves -- over this repo's restatement of the reference's
// interface (integration/iface/); options beyond BenchmarkConfig travel in
// XecPluginOptions.
//   --stdout         CSV to stdout instead of -f
//   --raw-dir DIR    directory for a bare -f name (default ../results/raw/; created
//                    if missing; "" = the working directory)
#include <getopt.h>
#include <omp.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "runner.hpp"
#include "xec_plugin_options.hpp"
#include "xorec_hip_bm.hpp"
#include "xorec_hip_multi_bm.hpp"

namespace {

const char* kName = "XOR-EC (HIP gfx950)";
const char* kNameMulti = "XOR-EC (HIP gfx950, multi-device)";

size_t parse_size(const char* s) {
  char* end = nullptr;
  unsigned long long v = std::strtoull(s, &end, 0);
  switch (end && *end ? *end : 0) {
    case 'K': case 'k': v <<= 10; break;
    case 'M': v <<= 20; break;
    case 'G': case 'g': v <<= 30; break;
    default: break;
  }
  return static_cast<size_t>(v);
}

// get_arg_vector (benchmark_suite.cpp:75-83): comma split, lower case
std::vector<std::string> arg_vector(const char* s) {
  std::vector<std::string> out;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    std::transform(tok.begin(), tok.end(), tok.begin(),
                   [](unsigned char c) { return static_cast<char>(std::tolower(c)); });
    out.push_back(tok);
  }
  return out;
}

void usage() {
  std::printf(
      "usage: xec_bench -g xorec-hip[,xorec-hip-multi] [-f out.csv] [-a] [-i iters] [-w warmup]\n"
      "                 [-s simd,...]\n"
      "  -f, --file FILE        output CSV (must contain .csv; default results.csv)\n"
      "  -a, --append           append rows, no header (default: overwrite + header)\n"
      "  -i, --iterations N     timed iterations per config (default 10)\n"
      "  -w, --warmup N         warm-up iterations per config (default 0)\n"
      "  -g, --gpu LIST         GPU algorithms: xorec-hip, xorec-hip-multi\n"
      "  -c, --cpu LIST         CPU algorithms: none in this build\n"
      "  -s, --simd LIST        scalar,sse2,avx2,avx512 (CPU variants only; no effect)\n"
      "  -h, --help\n"
      "extensions: --message B --block B --data K --parity M --lost L | --sweep FILE\n"
      "            --threads N --device D --devices LIST --seed S --sync MODE\n"
      "            --host-validation --stdout --raw-dir DIR\n"
      "without config options -g runs the reference's GPU sweep (get_gpu_configs)\n");
}

[[noreturn]] void fail(const std::string& msg) {
  std::cerr << "Error: " << msg << '\n';
  std::exit(EXIT_FAILURE);
}

// get_gpu_configs (benchmark_suite.cpp:252-277), same loop order
size_t parity_blocks(const BenchmarkConfig& c) {
  return std::get<0>(c.ec_params) - std::get<1>(c.ec_params);
}

std::vector<BenchmarkConfig> gpu_sweep(const BenchmarkConfig& base) {
  std::vector<BenchmarkConfig> out;
  for (size_t bs : VAR_BLOCK_SIZES)
    for (const auto& ec : VAR_EC_PARAMS) {
      const size_t m = std::get<0>(ec) - std::get<1>(ec);
      for (size_t lost : VAR_NUM_LOST_BLOCKS) {
        if (lost > m) continue;
        for (size_t gb : VAR_NUM_GPU_BLOCKS)
          for (size_t tpb : VAR_NUM_THREADS_PER_BLOCK) {
            BenchmarkConfig c = base;
            c.message_size = MESSAGE_SIZE;
            c.block_size = bs;
            c.ec_params = ec;
            c.num_lost_blocks = lost;
            c.num_cpu_threads = 0;  // as the reference's GPU configs
            c.gpu_computation = true;
            c.num_gpu_blocks = gb;
            c.threads_per_gpu_block = tpb;
            out.push_back(c);
          }
      }
    }
  return out;
}

}  // namespace

int main(int argc, char** argv) {
  enum { kMessage = 1000, kBlock, kData, kParity, kLost, kSweep, kThreads, kDevice, kSeed, kSync,
         kHostVal, kStdout, kDevices, kRawDir };
  const option long_options[] = {
      {"help", no_argument, nullptr, 'h'},
      {"file", required_argument, nullptr, 'f'},
      {"append", no_argument, nullptr, 'a'},
      {"iterations", required_argument, nullptr, 'i'},
      {"warmup", required_argument, nullptr, 'w'},
      {"cpu", required_argument, nullptr, 'c'},
      {"gpu", required_argument, nullptr, 'g'},
      {"simd", required_argument, nullptr, 's'},
      {"message", required_argument, nullptr, kMessage},
      {"block", required_argument, nullptr, kBlock},
      {"data", required_argument, nullptr, kData},
      {"parity", required_argument, nullptr, kParity},
      {"lost", required_argument, nullptr, kLost},
      {"sweep", required_argument, nullptr, kSweep},
      {"threads", required_argument, nullptr, kThreads},
      {"device", required_argument, nullptr, kDevice},
      {"seed", required_argument, nullptr, kSeed},
      {"sync", required_argument, nullptr, kSync},
      {"host-validation", no_argument, nullptr, kHostVal},
      {"stdout", no_argument, nullptr, kStdout},
      {"devices", required_argument, nullptr, kDevices},
      {"raw-dir", required_argument, nullptr, kRawDir},
      {nullptr, 0, nullptr, 0}};

  BenchmarkConfig base{};
  base.num_iterations = 10;        // NUM_ITERATIONS (benchmark_suite.cpp:30)
  base.num_warmup_iterations = 0;  // NUM_WARMUP_ITERATIONS (:31)
  base.gpu_computation = true;
  base.num_gpu_blocks = VAR_NUM_GPU_BLOCKS[0];
  base.threads_per_gpu_block = VAR_NUM_THREADS_PER_BLOCK[0];
  base.num_cpu_threads = static_cast<size_t>(omp_get_max_threads());
  XecPluginOptions opt;
  opt.seeded = true;  // reproducible unless --host-validation asks for the reference's clock
  // single-config defaults: BASELINE.json configs[2] (k=16+1, 1 MiB blocks,
  // 256 stripes = 4 GiB message, 1 lost block per stripe)
  BenchmarkConfig single = base;
  size_t k = 16, m = 1;
  single.block_size = 1u << 20;
  single.message_size = 256ull * 16 * (1u << 20);
  single.num_lost_blocks = 1;
  bool single_mode = false, overwrite = true, to_stdout = false;
  std::vector<std::string> algorithms;  // selected GPU algorithms, in -g order
  std::string out_file = "results.csv", sweep;
  std::string raw_dir = "../results/raw/";  // RAW_DIR, benchmark_suite.cpp:27

  int c, idx = 0;
  while ((c = getopt_long(argc, argv, "hf:ai:w:c:g:s:", long_options, &idx)) != -1) {
    switch (c) {
      case 'h': usage(); return EXIT_SUCCESS;
      case 'f':
        out_file = optarg;
        if (out_file.find(".csv") == std::string::npos) fail("Output file must have .csv extension.");
        break;
      case 'a': overwrite = false; break;
      case 'i':
        base.num_iterations = std::atoi(optarg);
        if (base.num_iterations <= 0) fail("Number of iterations must be positive.");
        break;
      case 'w':
        base.num_warmup_iterations = std::atoi(optarg);
        if (base.num_warmup_iterations < 0) fail("Number of warmup iterations must be non-negative.");
        break;
      case 'c':
        for (const auto& a : arg_vector(optarg))
          fail("Invalid CPU algorithm: " + a + " (this build carries the XOR-EC HIP path only)");
        break;
      case 'g':
        for (const auto& a : arg_vector(optarg)) {
          if (a != "xorec-hip" && a != "xorec-hip-multi") fail("Invalid GPU algorithm: " + a);
          if (std::find(algorithms.begin(), algorithms.end(), a) == algorithms.end())
            algorithms.push_back(a);
        }
        break;
      case 's':
        for (const auto& a : arg_vector(optarg))
          if (a != "scalar" && a != "sse2" && a != "avx2" && a != "avx512")
            fail("Invalid SIMD version: " + a);
        break;
      case kMessage: single.message_size = parse_size(optarg); single_mode = true; break;
      case kBlock: single.block_size = parse_size(optarg); single_mode = true; break;
      case kData: k = parse_size(optarg); single_mode = true; break;
      case kParity: m = parse_size(optarg); single_mode = true; break;
      case kLost: single.num_lost_blocks = parse_size(optarg); single_mode = true; break;
      case kSweep: sweep = optarg; break;
      case kThreads: base.num_cpu_threads = parse_size(optarg); break;
      case kDevice: opt.device = std::atoi(optarg); break;
      case kSeed: opt.seed = parse_size(optarg); break;
      case kSync: opt.sync_mode = std::atoi(optarg); break;
      case kHostVal: opt.seeded = false; opt.host_check = true; break;
      case kStdout: to_stdout = true; break;
      case kRawDir: raw_dir = optarg; break;
      case kDevices:
        opt.devices.clear();
        for (const auto& d : arg_vector(optarg)) {
          char* end = nullptr;
          const long v = std::strtol(d.c_str(), &end, 10);
          if (d.empty() || *end != '\0' || v < 0) fail("Invalid device: " + d);
          opt.devices.push_back(static_cast<int>(v));
        }
        break;
      default: usage(); return EXIT_FAILURE;
    }
  }
  if (algorithms.empty())
    fail("No benchmarks selected. Use --gpu xorec-hip (or xorec-hip-multi) to select one.");

  std::vector<BenchmarkConfig> cfgs;
  auto with_base = [&](BenchmarkConfig x) {
    x.num_iterations = base.num_iterations;
    x.num_warmup_iterations = base.num_warmup_iterations;
    return x;
  };
  if (!sweep.empty()) {
    std::ifstream in(sweep);
    if (!in) fail("cannot open " + sweep);
    std::string line;
    while (std::getline(in, line)) {
      if (line.empty() || line[0] == '#') continue;
      unsigned long long ms, b, kk, mm, l;
      if (std::sscanf(line.c_str(), "%llu %llu %llu %llu %llu", &ms, &b, &kk, &mm, &l) != 5) continue;
      BenchmarkConfig x = with_base(base);
      x.message_size = ms;
      x.block_size = b;
      x.ec_params = {kk + mm, kk};
      x.num_lost_blocks = l;
      cfgs.push_back(x);
    }
  } else if (single_mode) {
    single.ec_params = {k + m, k};
    cfgs.push_back(with_base(single));
  } else {
    cfgs = gpu_sweep(base);
  }
  for (const auto& x : cfgs) {
    if (x.num_lost_blocks > parity_blocks(x)) {
      // the reference prints and exits (utils.cpp:102-105)
      std::fprintf(stderr, "lost blocks per stripe (%zu) must be <= parity blocks (%zu)\n",
                   x.num_lost_blocks, parity_blocks(x));
      return 2;
    }
  }
  try {
    std::ofstream f;
    std::ostream* os = &std::cout;
    if (!to_stdout) {
      // a bare name goes to the raw-results directory (benchmark_suite.cpp:346)
      std::string path = out_file;
      if (out_file.find('/') == std::string::npos && !raw_dir.empty()) {
        std::error_code ec;
        std::filesystem::create_directories(raw_dir, ec);
        path = (std::filesystem::path(raw_dir) / out_file).string();
      }
      f.open(path, overwrite ? std::ios::out : std::ios::app);
      if (!f.is_open()) fail("Error opening file: " + path);
      os = &f;
    }
    // CSVReporter (csv_reporter.cpp:11-19): header only when overwriting
    if (overwrite) xec::write_csv_header(*os);
    int rc = 0;
    size_t n = 0;
    for (const auto& alg : algorithms) {
      const bool multi = alg == "xorec-hip-multi";
      for (const auto& x : cfgs) {
        xec::RunResult r = multi ? xec::run_generic<XorecBenchmarkHipMulti>(kNameMulti, x, opt)
                                 : xec::run_generic<XorecBenchmarkHip>(kName, x, opt);
        xec::write_csv_row(*os, r, x);
        os->flush();
        std::fprintf(stderr,
                     "[%zu/%zu] %s bs=%zu EC=(%zu/%zu) lost=%zu enc %.1f Gbit/s dec %.1f Gbit/s %s\n",
                     ++n, cfgs.size() * algorithms.size(), alg.c_str(), x.block_size,
                     std::get<0>(x.ec_params), std::get<1>(x.ec_params), x.num_lost_blocks,
                     r.encode.tp_mean, r.decode.tp_mean, r.err_msg.c_str());
        if (!r.err_msg.empty()) rc = 1;
      }
    }
    return rc;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "xec_bench: %s\n", e.what());
    return 3;
  }
}
