// runner.hpp -- timing harness with the reference's BM_generic semantics
// (src/benchmark/abstract_runner.hpp:36-150), without Google Benchmark:
//   warm-up x W: setup, encode, simulate_data_loss, decode
//   per iteration: setup | t encode | simulate_data_loss | t decode | validate
// encode/decode each end in a stream synchronise inside the plugin, so the
// steady_clock brackets cover the whole device work of that call.
// Throughput is the reference's: message bits / t_ns = Gbit/s
// (abstract_runner.hpp:66-68).  CSV rows use the reference's 20-column schema
// (src/reporters/csv_reporter.cpp:25-99), so results/raw tooling reads them.
#pragma once

#include <chrono>
#include <cmath>
#include <cstdio>
#include <numeric>
#include <ostream>
#include <string>
#include <vector>

#include "abstract_bm.hpp"           // the plugin interface (integration/iface/)
#include "xec_plugin_options.hpp"

namespace xec {

struct Stats {
  double t_mean = 0, t_stddev = 0, tp_mean = 0, tp_stddev = 0;
};

struct RunResult {
  std::string name;
  std::string err_msg;
  int iterations = 0;
  Stats encode, decode;
};

inline Stats compute_stats(const std::vector<double>& t_ns, size_t data_bytes) {
  Stats s;
  const double n = static_cast<double>(t_ns.size());
  if (t_ns.empty()) return s;
  s.t_mean = std::accumulate(t_ns.begin(), t_ns.end(), 0.0) / n;
  std::vector<double> tp;
  for (double t : t_ns) tp.push_back(static_cast<double>(data_bytes) * 8.0 / t);
  s.tp_mean = std::accumulate(tp.begin(), tp.end(), 0.0) / n;
  if (t_ns.size() > 1) {
    double vt = 0, vp = 0;
    for (size_t i = 0; i < t_ns.size(); ++i) {
      vt += (t_ns[i] - s.t_mean) * (t_ns[i] - s.t_mean);
      vp += (tp[i] - s.tp_mean) * (tp[i] - s.tp_mean);
    }
    s.t_stddev = std::sqrt(vt / (n - 1));
    s.tp_stddev = std::sqrt(vp / (n - 1));
  }
  return s;
}

template <typename Bench>
RunResult run_generic(const std::string& name, const ::BenchmarkConfig& cfg,
                      const XecPluginOptions& opt) {
  using clock = std::chrono::steady_clock;
  RunResult r;
  r.name = name;
  Bench bench(cfg, opt);
  ::AbstractBenchmark& b = bench;  // driven through the interface only, as BM_generic
  for (int i = 0; i < cfg.num_warmup_iterations; ++i) {
    b.setup();
    b.encode();
    b.simulate_data_loss();
    b.decode();
  }
  std::vector<double> enc, dec;
  for (int i = 0; i < cfg.num_iterations; ++i) {
    b.setup();
    auto t0 = clock::now();
    int rc = b.encode();
    auto t1 = clock::now();
    b.simulate_data_loss();
    auto t2 = clock::now();
    rc |= b.decode();
    auto t3 = clock::now();
    if (rc != 0 && r.err_msg.empty()) r.err_msg = "Codec Failure";
    if (!b.check_for_corruption() && r.err_msg.empty()) r.err_msg = "Corruption Detected";
    enc.push_back(std::chrono::duration<double, std::nano>(t1 - t0).count());
    dec.push_back(std::chrono::duration<double, std::nano>(t3 - t2).count());
    ++r.iterations;
  }
  r.encode = compute_stats(enc, cfg.message_size);
  r.decode = compute_stats(dec, cfg.message_size);
  return r;
}

inline void write_csv_header(std::ostream& os) {
  os << "name,err_msg,iterations,warmup_iterations,gpu_computation,gpu_blocks,threads_per_block,"
        "message_size_B,block_size_B,EC,lost_blocks,cpu_threads,encode_time_ns,"
        "encode_time_ns_stddev,encode_throughput_Gbps,encode_throughput_Gbps_stddev,"
        "decode_time_ns,decode_time_ns_stddev,decode_throughput_Gbps,"
        "decode_throughput_Gbps_stddev\n";
}

inline void write_csv_row(std::ostream& os, const RunResult& r, const ::BenchmarkConfig& c) {
  os << '"' << r.name << "\"," << r.err_msg << ',' << r.iterations << ','
     << c.num_warmup_iterations << ',' << (c.gpu_computation ? 1 : 0) << ',' << c.num_gpu_blocks
     << ',' << c.threads_per_gpu_block << ',' << c.message_size << ',' << c.block_size << ",\"("
     << std::get<0>(c.ec_params) << '/' << std::get<1>(c.ec_params) << ")\","
     << c.num_lost_blocks << ',' << c.num_cpu_threads << ',' << r.encode.t_mean << ','
     << r.encode.t_stddev << ',' << r.encode.tp_mean << ',' << r.encode.tp_stddev << ','
     << r.decode.t_mean << ',' << r.decode.t_stddev << ',' << r.decode.tp_mean << ','
     << r.decode.tp_stddev << '\n';
}

}  // namespace xec
