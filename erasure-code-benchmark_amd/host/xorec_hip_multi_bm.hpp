// xorec_hip_multi_bm.hpp -- the XOR-EC plugin over several MI355X in ONE
// process: the batch's stripes are cut into contiguous ranges, one per device
// (stripes are independent, xorec_bm.cpp:30 and
// xorec_gpu_cmp.cu:135-144, so no data crosses between devices and no
// collective is needed).  Each device holds its own data / parity / scratch
// slice in its HBM and has its own stream; encode() and decode() launch on
// every device and then wait for all of them, so the harness's clock around
// the call is the wall time from the first launch to the last completion
// across the devices.
//
// The same five virtuals and batch layout as XorecBenchmarkHip (and the
// reference's XorecBenchmarkGpuCmp, xorec_gpu_cmp_bm.cpp): a stripe's bytes
// sit at the same offsets inside its device's slice as they would in one
// buffer, validation payloads and erasure draws are seeded by the GLOBAL
// block / stripe index, so a batch gives the same bytes and the same losses
// on one device or on eight; decode() is all-or-nothing over the whole batch,
// so a failed decode leaves the same bytes too.  config.devices lists the devices (repeats
// allowed: two slices on one device exercise the sharding on a one-GPU box);
// empty = every visible device.
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <vector>

#include "abstract_bm.hpp"
#include "shard_pool.hpp"

namespace xec {

class XorecBenchmarkHipMulti : public AbstractBenchmark {
 public:
  explicit XorecBenchmarkHipMulti(const BenchmarkConfig& config);
  ~XorecBenchmarkHipMulti() noexcept override;
  XorecBenchmarkHipMulti(const XorecBenchmarkHipMulti&) = delete;
  XorecBenchmarkHipMulti& operator=(const XorecBenchmarkHipMulti&) = delete;

  void setup() noexcept override;
  int encode() noexcept override;
  int decode() noexcept override;
  void simulate_data_loss() noexcept override;
  bool check_for_corruption() const noexcept override;

  size_t shards() const { return m_shards.size(); }
  // Stripe range [first, first + count) and device of shard i.
  size_t shard_first(size_t i) const { return m_shards[i].first; }
  size_t shard_count(size_t i) const { return m_shards[i].count; }
  int shard_device(size_t i) const { return m_shards[i].device; }
  // Copies shard i's data / parity slice to host memory (tests).
  bool read_shard(size_t i, uint8_t* h_data, uint8_t* h_parity) const noexcept;

  // Config 5's exchange in one process: the batch starts
  // in the HBM of `root` (S*k*bs bytes, the reference layout) and every
  // shard's stripe range is copied to its device with hipMemcpyPeerAsync --
  // xGMI DMA between GPUs, a device copy when shard and root share one --
  // all shards at once on their own streams; returns when every copy has
  // landed (0, or -1 on a HIP error).  Peer access to root is enabled where
  // the devices allow it.  gather_parity_to is the inverse for the parity
  // (S*m*bs bytes on root).  No collective: stripes are independent.
  int scatter_from(const uint8_t* d_root_data, int root) noexcept;
  int gather_parity_to(uint8_t* d_root_parity, int root) noexcept;

 protected:
  void m_write_data_buffer() noexcept override;

 private:
  struct Shard {
    int device = 0;
    hipStream_t stream = nullptr;
    size_t first = 0, count = 0;  // global stripe range
    Buffer data{nullptr, nullptr};      // device count*k*bs
    Buffer parity{nullptr, nullptr};    // device count*m*bs
    Buffer d_bitmap{nullptr, nullptr};  // device scratch for xec_decode, count*(k+m)
    Buffer d_erase{nullptr, nullptr};   // device copy of the erasure bitmap slice
    Buffer d_bad{nullptr, nullptr};     // device counter of corrupted blocks
  };
  // Runs fn(shard) on every shard with its device current, then waits for
  // every stream; false if any call or wait failed.
  template <typename F>
  bool each(F&& fn) const noexcept;

  // m_block_bitmap: pinned host S*(k+m) for the whole batch (base-class
  // member, replaced in the constructor); m_data_buf / m_parity_buf unused.
  std::vector<Shard> m_shards;
  std::unique_ptr<ShardPool> m_pool;  // decode(): one thread per shard (shard_pool.hpp)
  bool enable_peer(int root) noexcept;
  void destroy_streams() noexcept;  // synchronise and destroy every shard's stream
  int m_last_status = 0;
};

}  // namespace xec
