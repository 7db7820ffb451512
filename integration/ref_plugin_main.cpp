// ref_plugin_main.cpp -- drives XorecBenchmarkHip (or, with the argument
// "multi", XorecBenchmarkHipMulti over XEC_DEVICES / every visible device)
// through one iteration of the reference's timing loop (BM_generic, src/benchmark/abstract_runner.hpp:
// 97-121: setup, encode, simulate_data_loss, decode, check_for_corruption)
// through the AbstractBenchmark interface only.  Built by integration/Makefile
// to show that the plugin links against libxec_hip.so together with the
// reference's own abstract_bm.cpp and utils.cpp; it is compiled and linked in
// the container, never shipped.
#include <cstdio>
#include <cstring>
#include <memory>

#include "xorec_hip_bm.hpp"
#include "xorec_hip_multi_bm.hpp"

int main(int argc, char** argv) {
  const bool multi = argc > 1 && std::strcmp(argv[1], "multi") == 0;
  BenchmarkConfig config{};
  config.message_size = 8 MiB;
  config.block_size = 64 KiB;
  config.ec_params = ECTuple(17, 16);  // (total, data) blocks: 16 data + 1 parity
  config.num_lost_blocks = 1;
  config.num_cpu_threads = 1;
  config.num_iterations = 1;
  config.num_warmup_iterations = 0;
  config.gpu_computation = true;

  std::unique_ptr<AbstractBenchmark> bench;
  if (multi)
    bench = std::make_unique<XorecBenchmarkHipMulti>(config);
  else
    bench = std::make_unique<XorecBenchmarkHip>(config);
  bench->setup();
  const int enc = bench->encode();
  bench->simulate_data_loss();
  const int dec = bench->decode();
  const bool ok = bench->check_for_corruption();
  std::printf("encode %d decode %d valid %d\n", enc, dec, ok ? 1 : 0);
  return (enc == 0 && dec == 0 && ok) ? 0 : 1;
}
