// xec_bench.cpp -- command-line harness: the reference's "xorec-gpu" benchmark
// (BM_XOREC_GPU_CMP, src/benchmark/runners.cpp:43-45) re-registered as
// "xorec-hip", one CSV row per configuration in the reference's schema.
//
//   xec_bench [-s message_bytes] [-b block_bytes] [-k data] [-m parity]
//             [-l lost_per_stripe] [-i iterations] [-w warmup] [-t cpu_threads]
//             [-d device] [-r seed] [-o out.csv] [--no-header] [-f sweep_file]
//             [-y sync_mode: 0 default, 1 spin, 2 yield, 3 blocking]
//             [-V: validation payload on the host + copies, as the reference]
// -f runs every line "message_bytes block_bytes k m lost" of sweep_file in
// this process (one CSV row each), like the reference's config cross-product
// (benchmark_suite.cpp:220-318).
// Sizes accept K/M/G suffixes (binary).  Defaults: BASELINE.json configs[2]
// (k=16+1, 1 MiB blocks, 256 stripes = 4 GiB message), 1 lost block, 10
// iterations, 0 warm-up (the reference's defaults, benchmark_suite.cpp:30-31).
#include <omp.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "runner.hpp"
#include "xorec_hip_bm.hpp"

namespace {

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

void usage() {
  std::fprintf(stderr,
               "usage: xec_bench [-s message_bytes] [-b block_bytes] [-k data] [-m parity]\n"
               "                 [-l lost] [-i iters] [-w warmup] [-t threads] [-d device]\n"
               "                 [-r seed] [-o out.csv] [--no-header] [-f sweep_file]\n"
               "                 [-y sync_mode] [-V]\n");
}

}  // namespace

int main(int argc, char** argv) {
  xec::BenchmarkConfig cfg;
  size_t k = 16, m = 1;
  cfg.block_size = 1 << 20;
  cfg.message_size = 256ull * 16 * (1 << 20);
  cfg.num_lost_blocks = 1;
  cfg.num_cpu_threads = static_cast<size_t>(omp_get_max_threads());
  std::string out, sweep;
  bool header = true;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&]() -> const char* {
      if (i + 1 >= argc) { usage(); std::exit(2); }
      return argv[++i];
    };
    if (a == "-s") cfg.message_size = parse_size(val());
    else if (a == "-b") cfg.block_size = parse_size(val());
    else if (a == "-k") k = parse_size(val());
    else if (a == "-m") m = parse_size(val());
    else if (a == "-l") cfg.num_lost_blocks = parse_size(val());
    else if (a == "-i") cfg.num_iterations = std::atoi(val());
    else if (a == "-w") cfg.num_warmup_iterations = std::atoi(val());
    else if (a == "-t") cfg.num_cpu_threads = parse_size(val());
    else if (a == "-d") cfg.device_id = std::atoi(val());
    else if (a == "-r") cfg.seed = parse_size(val());
    else if (a == "-o") out = val();
    else if (a == "--no-header") header = false;
    else if (a == "-f") sweep = val();
    else if (a == "-y") cfg.sync_mode = std::atoi(val());
    else if (a == "-V") cfg.host_validation = true;
    else if (a == "-h" || a == "--help") { usage(); return 0; }
    else { usage(); return 2; }
  }
  std::vector<xec::BenchmarkConfig> cfgs;
  if (sweep.empty()) {
    cfg.ec_params = {k + m, k};
    cfgs.push_back(cfg);
  } else {
    std::ifstream in(sweep);
    if (!in) {
      std::fprintf(stderr, "cannot open %s\n", sweep.c_str());
      return 2;
    }
    std::string line;
    while (std::getline(in, line)) {
      if (line.empty() || line[0] == '#') continue;
      unsigned long long ms, b, kk, mm, l;
      if (std::sscanf(line.c_str(), "%llu %llu %llu %llu %llu", &ms, &b, &kk, &mm, &l) != 5) continue;
      xec::BenchmarkConfig c = cfg;
      c.message_size = ms;
      c.block_size = b;
      c.ec_params = {kk + mm, kk};
      c.num_lost_blocks = l;
      cfgs.push_back(c);
    }
  }
  for (const auto& c : cfgs) {
    if (c.num_lost_blocks > xec::parity_blocks(c)) {
      // the reference prints and exits (utils.cpp:102-105)
      std::fprintf(stderr, "lost blocks per stripe (%zu) must be <= parity blocks (%zu)\n",
                   c.num_lost_blocks, xec::parity_blocks(c));
      return 2;
    }
  }
  try {
    std::ofstream f;
    std::ostream* os = &std::cout;
    if (!out.empty()) {
      f.open(out, std::ios::app);
      os = &f;
    }
    if (header) xec::write_csv_header(*os);
    int rc = 0;
    for (const auto& c : cfgs) {
      xec::RunResult r = xec::run_generic<xec::XorecBenchmarkHip>("XOR-EC (HIP gfx950)", c);
      xec::write_csv_row(*os, r, c);
      os->flush();
      if (!r.err_msg.empty()) rc = 1;
    }
    return rc;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "xec_bench: %s\n", e.what());
    return 3;
  }
}
