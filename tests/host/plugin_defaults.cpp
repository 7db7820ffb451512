// plugin_defaults.cpp -- a CPU plugin that overrides ONLY setup / encode /
// decode, run through the harness loop (host/runner.hpp): the base class's
// default simulate_data_loss, check_for_corruption and m_write_data_buffer
// (integration/iface/abstract_bm.cpp, restating abstract_bm.cpp:20-60) must make it work,
// as the reference's CPU plugins rely on (e.g. xorec_bm.cpp:6-58).  The codec
// here is the oracle's C restatement (test infrastructure).  A second plugin
// whose decode does nothing must be caught by the default corruption check.
#include <cstdio>
#include <cstring>
#include <string>

#include "runner.hpp"
#include "xorec_oracle.h"

namespace {

class CpuXorecPlugin : public AbstractBenchmark {
 public:
  explicit CpuXorecPlugin(const BenchmarkConfig& c, const XecPluginOptions& = {})
      : AbstractBenchmark(c) {}
  void setup() noexcept override {
    std::memset(m_block_bitmap.get(), 1, m_chunks * m_chunk_tot_blocks);
    m_write_data_buffer();
  }
  int encode() noexcept override {
    return xo_encode_batch(m_data_buf.get(), m_parity_buf.get(), m_chunks, m_block_size,
                           m_chunk_data_blocks, m_chunk_parity_blocks, 1);
  }
  int decode() noexcept override {
    return xo_decode_batch(m_data_buf.get(), m_parity_buf.get(), m_chunks, m_block_size,
                           m_chunk_data_blocks, m_chunk_parity_blocks, m_block_bitmap.get(), 1);
  }
};

class NoDecodePlugin : public CpuXorecPlugin {
 public:
  using CpuXorecPlugin::CpuXorecPlugin;
  int decode() noexcept override { return 0; }
};

int failures = 0;

void expect(bool ok, const std::string& what) {
  if (!ok) {
    std::printf("FAIL %s\n", what.c_str());
    ++failures;
  }
}

BenchmarkConfig cfg(size_t msg, size_t bs, size_t k, size_t m, size_t lost) {
  BenchmarkConfig c{};
  c.message_size = msg;
  c.block_size = bs;
  c.ec_params = {k + m, k};
  c.num_lost_blocks = lost;
  c.num_iterations = 3;
  c.num_warmup_iterations = 1;
  c.gpu_computation = false;
  return c;
}

}  // namespace

int main() {
  const size_t shapes[][5] = {{1 << 20, 1024, 8, 4, 4}, {1 << 20, 4096, 16, 1, 1},
                              {1 << 20, 2048, 32, 8, 8}, {1 << 20, 1024, 8, 4, 0},
                              {3 << 19, 512, 12, 4, 2}};
  for (const auto& s : shapes) {
    const auto c = cfg(s[0], s[1], s[2], s[3], s[4]);
    const std::string tag = std::to_string(s[2]) + "+" + std::to_string(s[3]) + " lost " +
                            std::to_string(s[4]);
    auto r = xec::run_generic<CpuXorecPlugin>("cpu", c, XecPluginOptions{});
    expect(r.err_msg.empty(), "defaults, " + tag + ": " + r.err_msg);
    expect(r.iterations == 3, "iterations, " + tag);
    if (s[4] > 0) {
      auto bad = xec::run_generic<NoDecodePlugin>("nodecode", c, XecPluginOptions{});
      expect(bad.err_msg == "Corruption Detected", "default check catches a skipped decode, " + tag);
    }
  }
  // the default erasure draw: exactly `lost` zero bitmap bytes per stripe,
  // at most one per parity class (select_lost_blocks, utils.cpp:100-127)
  struct Probe : CpuXorecPlugin {
    using CpuXorecPlugin::CpuXorecPlugin;
    bool ok(size_t lost) {
      setup();
      simulate_data_loss();
      for (size_t c = 0; c < m_chunks; ++c) {
        const uint8_t* b = m_block_bitmap.get() + c * m_chunk_tot_blocks;
        size_t zeros = 0;
        std::string cls(m_chunk_parity_blocks, 0);
        for (size_t i = 0; i < m_chunk_tot_blocks; ++i) {
          if (b[i]) continue;
          ++zeros;
          const size_t j = i < m_chunk_data_blocks ? i % m_chunk_parity_blocks : i - m_chunk_data_blocks;
          if (cls[j]++) return false;
          // a lost block is zeroed
          const uint8_t* blk = i < m_chunk_data_blocks
                                   ? m_data_buf.get() + c * m_chunk_data_size + i * m_block_size
                                   : m_parity_buf.get() + c * m_chunk_parity_size +
                                         (i - m_chunk_data_blocks) * m_block_size;
          for (size_t x = 0; x < m_block_size; ++x)
            if (blk[x]) return false;
        }
        if (zeros != lost) return false;
      }
      return true;
    }
  };
  Probe p(cfg(1 << 20, 1024, 16, 8, 8));
  expect(p.ok(8), "default simulate_data_loss draws 8 per stripe, one per class, zeroed");
  if (failures == 0) std::printf("plugin_defaults ok\n");
  return failures ? 1 : 0;
}
