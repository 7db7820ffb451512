// xorec_hip_multi_bm.hpp -- the MI355X XOR-EC plugin over SEVERAL GPUs of one
// node in one process (BASELINE.json configs[4]), implementing the reference's
// plugin interface (src/algorithms/abstract_bm.hpp:18-88) as a maintainer adds
// it to src/algorithms/ next to XorecBenchmarkGpuCmp (xorec_gpu_cmp_bm.hpp:1-23).
// One source, two builds: see xorec_hip_bm.hpp.
//
// BenchmarkConfig is used as the reference defines it: no new field.  The
// devices come from XecPluginOptions::devices, else the environment variable
// XEC_DEVICES (comma-separated HIP device ids, repeats allowed: "0,0" cuts the
// batch into two slices on one GPU), else every visible device.
//
// The batch's stripes are cut into contiguous ranges, one per device (stripes
// are independent: xorec_bm.cpp:30, xorec_gpu_cmp.cu:135-144), each range's
// data / parity / scratch in its device's HBM, each device with its own
// stream; a stripe sits at the same offset inside its range as in one
// buffer.  encode() / decode() launch on every device, then wait for all, so
// BM_generic's clock (abstract_runner.hpp:104-112) spans first launch to last
// completion.  decode() is all-or-nothing over the WHOLE batch, as the
// reference's GPU decode (xorec_gpu_cmp.cu:75-81): every range's bitmap is
// checked before any device launches; each range's scan and launch run on
// its own thread (shard_pool.hpp), so no device waits for another's scan.
#ifndef XOREC_HIP_MULTI_BM_HPP
#define XOREC_HIP_MULTI_BM_HPP

#include <memory>
#include <vector>

#include "abstract_bm.hpp"
#include "hip_buffers.hpp"
#include "xec.h"
#include "xec_plugin_options.hpp"

namespace xec_hip {
class ShardPool;
}

class XorecBenchmarkHipMulti : public AbstractBenchmark {
public:
  explicit XorecBenchmarkHipMulti(const BenchmarkConfig& config);
  XorecBenchmarkHipMulti(const BenchmarkConfig& config, const XecPluginOptions& options);
  ~XorecBenchmarkHipMulti() noexcept override;
  XorecBenchmarkHipMulti(const XorecBenchmarkHipMulti&) = delete;
  XorecBenchmarkHipMulti& operator=(const XorecBenchmarkHipMulti&) = delete;

  void setup() noexcept override;
  int encode() noexcept override;
  int decode() noexcept override;
  void simulate_data_loss() noexcept override;
  bool check_for_corruption() const noexcept override;

  // Config 5's exchange (no reference counterpart: the reference is one GPU):
  // the batch starts in `root`'s HBM (the reference layout, m_chunks stripes)
  // and each range is copied to its device over xGMI (hipMemcpyPeerAsync; a
  // device copy where shard and root share one), all shards at once on their
  // own streams; gather_parity_to is the inverse for the parity.  Return
  // when every copy has landed; 0 or -1.  No collective: stripes are
  // independent.
  int scatter_from(const uint8_t* d_root_data, int root) noexcept;
  int gather_parity_to(uint8_t* d_root_parity, int root) noexcept;
  // How shard i's device reached the root in the last scatter_from /
  // gather_parity_to (hip_buffers.hpp PeerAccess): kEnabled = peer DMA,
  // kStaged = the pair has no peer access and the runtime staged the copies
  // (reported as "staged", peer_path.hpp), kSameDevice = a device copy;
  // kError before any exchange.
  xec_hip::PeerAccess shard_peer_access(size_t i) const noexcept { return m_shards[i].peer; }

  // Shards and diagnostics for the harness and tests.
  size_t num_shards() const noexcept { return m_shards.size(); }
  size_t shard_first(size_t i) const noexcept { return m_shards[i].first; }
  size_t shard_count(size_t i) const noexcept { return m_shards[i].count; }
  int shard_device(size_t i) const noexcept { return m_shards[i].device; }
  // Copies shard i's data / parity range to host memory; false on failure.
  bool read_shard(size_t i, uint8_t* h_data, uint8_t* h_parity) const noexcept;
  int last_status() const noexcept { return m_last_status; }
  size_t lost_data_blocks() const noexcept;

protected:
  void m_write_data_buffer() noexcept override;

private:
  using DevBuf = std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>>;
  struct Shard {
    int device = 0;
    hipStream_t stream = nullptr;
    size_t first = 0, count = 0;  ///< global stripe range
    DevBuf data{nullptr, nullptr};      ///< count * k * bs
    DevBuf parity{nullptr, nullptr};    ///< count * m * bs
    DevBuf d_bitmap{nullptr, nullptr};  ///< xec_decode scratch, count * (k + m)
    DevBuf d_erase{nullptr, nullptr};   ///< device copy of the erasure bitmap slice
    DevBuf d_bad{nullptr, nullptr};     ///< device count of invalid blocks
    DevBuf h_stage{nullptr, nullptr};   ///< pinned copy of the range (host payload / check)
    xec_hip::PeerAccess peer = xec_hip::PeerAccess::kError;  ///< to the last exchange's root
  };

  // Runs fn(shard) on every shard with its device current, then waits for
  // every stream; false if any call or wait failed.  The caller's current
  // device is restored.
  template <typename F>
  bool each(F&& fn) const noexcept;
  bool enable_peers(int root) noexcept;
  void destroy_streams() noexcept;

  XecPluginOptions m_opt;
  uint64_t m_round = 0;  ///< setup() count: a fresh seeded round per iteration
  std::vector<Shard> m_shards;
  std::unique_ptr<xec_hip::ShardPool> m_pool;  ///< decode(): one thread per shard
  int m_last_status = 0;
};

#endif  // XOREC_HIP_MULTI_BM_HPP
