// xorec_hip_multi_bm.cpp -- see xorec_hip_multi_bm.hpp.  Each method follows
// the XorecBenchmarkGpuCmp method it replaces (src/algorithms/
// xorec_gpu_cmp_bm.cpp), per device range, with the interface's utilities
// (utils.hpp) where that plugin uses them; codec calls are include/xec.h.
#include "xorec_hip_multi_bm.hpp"

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <sstream>
#include <string>

#include "hip_buffers.hpp"
#include "shard_pool.hpp"
#include "utils.hpp"

namespace {

// The device list: the options', else XEC_DEVICES ("0,1,2,...", repeats
// allowed), else every visible device.  BenchmarkConfig carries no device
// field (bm_config.hpp:25-43), so the list travels beside it.
std::vector<int> plugin_devices(const std::vector<int>& given) {
  const int visible = xec_hip::device_count();
  std::vector<int> devs = given;
  if (devs.empty()) {
    if (const char* env = std::getenv("XEC_DEVICES"); env != nullptr && *env != '\0') {
      std::stringstream ss(env);
      std::string tok;
      while (std::getline(ss, tok, ',')) {
        char* end = nullptr;
        const long d = std::strtol(tok.c_str(), &end, 10);
        if (tok.empty() || *end != '\0' || d < 0)
          throw_error("XorecBenchmarkHipMulti: bad device '" + tok + "' in XEC_DEVICES");
        devs.push_back(static_cast<int>(d));
      }
    } else {
      for (int d = 0; d < visible; ++d) devs.push_back(d);
    }
  }
  for (int d : devs)
    if (d < 0 || d >= visible)
      throw_error("XorecBenchmarkHipMulti: no HIP device " + std::to_string(d));
  if (devs.empty()) throw_error("XorecBenchmarkHipMulti: no HIP device");
  return devs;
}

void no_free(uint8_t*) {}

// The caller's current device, restored on scope exit.
struct DeviceRestore {
  int dev = xec_hip::current_device();
  ~DeviceRestore() {
    if (dev >= 0) (void)xec_hip::set_device(dev);
  }
};

}  // namespace

XorecBenchmarkHipMulti::XorecBenchmarkHipMulti(const BenchmarkConfig& config)
  : XorecBenchmarkHipMulti(config, XecPluginOptions{}) {}

// XorecBenchmarkGpuCmp ctor (xorec_gpu_cmp_bm.cpp:6-18), once per device range:
// the base class's host data / parity buffers are dropped (the batch lives in
// the devices' HBM) and the bitmap is pinned host memory every device reads.
XorecBenchmarkHipMulti::XorecBenchmarkHipMulti(const BenchmarkConfig& config,
                                               const XecPluginOptions& options)
  : AbstractBenchmark(config), m_opt(options) {
  const DeviceRestore restore;
  const std::vector<int> devs = plugin_devices(m_opt.devices);
  m_data_buf = std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>>(nullptr, no_free);
  m_parity_buf = std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>>(nullptr, no_free);
  uint8_t* bm = xec_hip::alloc_pinned(m_chunks * m_chunk_tot_blocks);
  if (bm == nullptr) throw_error("XorecBenchmarkHipMulti: hipHostMalloc failed");
  m_block_bitmap = std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>>(bm, xec_hip::free_pinned);
  // contiguous ranges, the first m_chunks % n one stripe longer
  // (xec/partition.py stripe_range)
  const size_t n = devs.size(), base = m_chunks / n, extra = m_chunks % n;
  m_shards.resize(n);
  auto dev_buf = [](size_t bytes) {
    uint8_t* p = xec_hip::alloc_device(bytes);
    if (p == nullptr) throw_error("XorecBenchmarkHipMulti: hipMalloc failed");
    return DevBuf(p, xec_hip::free_device);
  };
  try {
    for (size_t i = 0; i < n; ++i) {
      Shard& s = m_shards[i];
      s.device = devs[i];
      s.first = i * base + std::min(i, extra);
      s.count = base + (i < extra ? 1 : 0);
      if (!xec_hip::set_device(s.device)) throw_error("XorecBenchmarkHipMulti: bad device");
      (void)xec_hip::set_sync_mode(m_opt.sync_mode);  // before the context is active
      if (xec_init(s.device) != XEC_SUCCESS)  // also makes s.device current
        throw_error("XorecBenchmarkHipMulti: xec_init(" + std::to_string(s.device) + ") failed");
      s.stream = xec_hip::create_stream();
      if (s.stream == nullptr) throw_error("XorecBenchmarkHipMulti: hipStreamCreate failed");
      s.data = dev_buf(s.count * m_chunk_data_size);
      s.parity = dev_buf(s.count * m_chunk_parity_size);
      s.d_bitmap = dev_buf(s.count * m_chunk_tot_blocks);
      s.d_erase = dev_buf(s.count * m_chunk_tot_blocks);
      s.d_bad = dev_buf(sizeof(uint32_t));
      if (!m_opt.seeded || m_opt.host_check) {
        uint8_t* h = xec_hip::alloc_pinned(s.count * m_chunk_data_size);
        if (h == nullptr) throw_error("XorecBenchmarkHipMulti: hipHostMalloc failed");
        s.h_stage = DevBuf(h, xec_hip::free_pinned);
      }
    }
    m_pool = std::make_unique<xec_hip::ShardPool>(n);
  } catch (...) {
    // no destructor runs for a throwing constructor: the streams made so far
    // go here, the buffers with m_shards
    destroy_streams();
    throw;
  }
}

void XorecBenchmarkHipMulti::destroy_streams() noexcept {
  for (Shard& s : m_shards) {
    if (s.stream == nullptr || !xec_hip::set_device(s.device)) continue;
    (void)xec_hip::synchronize(s.stream);
    xec_hip::destroy_stream(s.stream);
    s.stream = nullptr;
  }
}

XorecBenchmarkHipMulti::~XorecBenchmarkHipMulti() noexcept {
  const DeviceRestore restore;
  m_pool.reset();  // join the workers before the streams they use go
  destroy_streams();
  // device buffers are released by their deleters after this body
}

template <typename F>
bool XorecBenchmarkHipMulti::each(F&& fn) const noexcept {
  const DeviceRestore restore;
  bool ok = true;
  for (const Shard& s : m_shards)  // launch everywhere first ...
    ok = xec_hip::set_device(s.device) && fn(s) && ok;
  for (const Shard& s : m_shards)  // ... then wait for every device
    ok = xec_hip::set_device(s.device) && xec_hip::synchronize(s.stream) && ok;
  return ok;
}

// xorec_gpu_cmp_bm.cpp:20-23
void XorecBenchmarkHipMulti::setup() noexcept {
  ++m_round;
  std::fill_n(m_block_bitmap.get(), m_chunks * m_chunk_tot_blocks, 1);
  m_write_data_buffer();
}

// xorec_gpu_cmp_bm.cpp:25-37 per device range: the reference's
// write_validation_pattern (utils.cpp:35-69) on the host, one copy per range.
// Seeded: written on each device, global data block b of round r from
// seed + (r << 32) + b -- the same bytes as the one-device plugin's.
void XorecBenchmarkHipMulti::m_write_data_buffer() noexcept {
  const uint64_t round_base = m_opt.seed + (m_round << 32);
  if (m_opt.seeded) {
    if (!each([&](const Shard& s) {
          return s.count == 0 ||
                 xec_write_validation_pattern(s.data.get(), s.count * m_chunk_data_blocks,
                                              m_block_size,
                                              round_base + s.first * m_chunk_data_blocks,
                                              s.stream) == XEC_SUCCESS;
        }))
      throw_error("XorecBenchmarkHipMulti: device payload failed");
    return;
  }
  for (const Shard& s : m_shards) {
    if (s.count == 0) continue;
    uint8_t* stage = s.h_stage.get();
    const long long blocks = static_cast<long long>(s.count * m_chunk_data_blocks);
    bool failed = false;
#pragma omp parallel for schedule(static) reduction(|| : failed)
    for (long long b = 0; b < blocks; ++b)
      failed = write_validation_pattern(stage + static_cast<size_t>(b) * m_block_size,
                                        m_block_size) != 0 || failed;
    if (failed) throw_error("Failed to write random checking packet.");
    const DeviceRestore restore;
    if (!xec_hip::set_device(s.device) ||
        !xec_hip::copy_to_device(s.data.get(), stage, s.count * m_chunk_data_size, s.stream) ||
        !xec_hip::synchronize(s.stream))
      throw_error("XorecBenchmarkHipMulti: data upload failed");
  }
}

// xorec_gpu_cmp_bm.cpp:39-52, on every range at once
int XorecBenchmarkHipMulti::encode() noexcept {
  int status = XEC_SUCCESS;
  const bool ok = each([&](const Shard& s) {
    const xec_status st = xec_encode(s.data.get(), s.parity.get(), s.count, m_block_size,
                                     m_chunk_data_blocks, m_chunk_parity_blocks, s.stream);
    if (st != XEC_SUCCESS && status == XEC_SUCCESS) status = st;
    return st == XEC_SUCCESS;
  });
  m_last_status = status;
  return ok ? 0 : -1;
}

// xorec_gpu_cmp_bm.cpp:54-69.  All-or-nothing over the WHOLE batch, like the
// one-device plugin and the reference's GPU decode (xorec_gpu_cmp.cu:75-81):
// each shard's thread (m_pool) first checks its slice of the host bitmap
// (xec_check_bitmap: is_recoverable per stripe, xorec_utils.hpp:160-175), then
// all meet (Rendezvous); if any stripe of any shard is unrecoverable no shard
// launches anything and the call fails, so the bytes after a failed decode do
// not depend on the device count.  Otherwise every shard decodes its slice
// (xec_decode: host scan, then the launch) on its own thread, so no device's
// launch waits for another's scan; then every stream is waited for.
// The library's tuning overrides are per thread (include/xec.h): the caller's
// are copied into every worker before its xec_decode, so all shards launch the
// shape the caller configured, not the workers' defaults.  Parity is read-only.
int XorecBenchmarkHipMulti::decode() noexcept {
  const size_t n = m_shards.size();
  std::vector<int> st(n, XEC_DEVICE_ERROR);
  xec_hip::Rendezvous all_recoverable(n);
  bool launched = false;  // every shard reached xec_decode (written by shard 0)
  xec_tuning tuning{};
  const bool tuned = xec_get_tuning(&tuning) == XEC_SUCCESS;
  m_pool->run([&](size_t i) {
    const Shard& s = m_shards[i];
    if (i != 0 && (!tuned || xec_set_tuning(&tuning) != XEC_SUCCESS)) {
      (void)all_recoverable.arrive(false);  // the others must not wait for this shard
      return;                               // st[i] stays XEC_DEVICE_ERROR
    }
    const uint8_t* bm = m_block_bitmap.get() + s.first * m_chunk_tot_blocks;
    int needs = 0;
    const xec_status check = xec_check_bitmap(bm, s.count, m_chunk_data_blocks,
                                              m_chunk_parity_blocks, &needs);
    const bool go = all_recoverable.arrive(check == XEC_SUCCESS);
    if (i == 0) launched = go;
    if (!go) {
      st[i] = check;  // this shard's own verdict (0 if only another shard failed)
      return;
    }
    const DeviceRestore restore;
    if (!xec_hip::set_device(s.device)) return;
    st[i] = xec_decode(s.data.get(), s.parity.get(), s.count, m_block_size, m_chunk_data_blocks,
                       m_chunk_parity_blocks, bm, s.d_bitmap.get(), s.stream);
  });
  const bool ok = !launched || each([](const Shard&) { return true; });  // wait for every stream
  int status = XEC_SUCCESS;
  for (int v : st)
    if (v != XEC_SUCCESS) {
      status = v;
      break;
    }
  m_last_status = status;
  return ok && static_cast<XorecResult>(status) == XorecResult::Success ? 0 : -1;
}

// xorec_gpu_cmp_bm.cpp:71-89: erasure sets drawn per GLOBAL stripe on the host
// (the reference's select_lost_blocks, utils.cpp:100-127; seeded:
// xec_select_lost_blocks, stripe c of round r from seed + (r << 32) + c, as
// the one-device plugin), zeroed on each device by one xec_erase kernel
// instead of a cudaMemset per lost block.
void XorecBenchmarkHipMulti::simulate_data_loss() noexcept {
  const size_t tot = m_chunk_tot_blocks;
  uint8_t* bm = m_block_bitmap.get();
  for (size_t c = 0; c < m_chunks; ++c) {
    if (m_opt.seeded) {
      if (xec_select_lost_blocks(m_chunk_data_blocks, m_chunk_parity_blocks, m_chunk_lost_blocks,
                                 bm + c * tot, m_opt.seed + (m_round << 32) + c) != XEC_SUCCESS)
        throw_error("XorecBenchmarkHipMulti: lost blocks must be <= parity blocks");
    } else {
      select_lost_blocks(m_chunk_data_blocks, m_chunk_parity_blocks, m_chunk_lost_blocks,
                         bm + c * tot);
    }
  }
  const bool ok = each([&](const Shard& s) {
    return s.count == 0 ||
           (xec_hip::copy_to_device(s.d_erase.get(), bm + s.first * tot, s.count * tot,
                                    s.stream) &&
            xec_erase(s.data.get(), s.parity.get(), s.count, m_block_size, m_chunk_data_blocks,
                      m_chunk_parity_blocks, s.d_erase.get(), s.stream) == XEC_SUCCESS);
  });
  if (!ok) throw_error("XorecBenchmarkHipMulti: erasure failed");
}

// xorec_gpu_cmp_bm.cpp:91-104: every data block's embedded checksum
// (validate_block, utils.cpp:72-97), checked on its device -- or, with
// host_check, on the host after a copy of each range.
bool XorecBenchmarkHipMulti::check_for_corruption() const noexcept {
  if (m_opt.host_check) {
    for (const Shard& s : m_shards) {
      if (s.count == 0) continue;
      const DeviceRestore restore;
      uint8_t* stage = s.h_stage.get();
      if (!xec_hip::set_device(s.device) ||
          !xec_hip::copy_to_host(stage, s.data.get(), s.count * m_chunk_data_size, s.stream) ||
          !xec_hip::synchronize(s.stream))
        return false;
      const long long blocks = static_cast<long long>(s.count * m_chunk_data_blocks);
      long long bad = 0;
#pragma omp parallel for schedule(static) reduction(+ : bad)
      for (long long b = 0; b < blocks; ++b)
        bad += validate_block(stage + static_cast<size_t>(b) * m_block_size, m_block_size) ? 0 : 1;
      if (bad != 0) return false;
    }
    return true;
  }
  std::vector<uint32_t> bad(m_shards.size(), 0);
  size_t i = 0;
  const bool ok = each([&](const Shard& s) {
    uint32_t* h_bad = &bad[i++];
    if (s.count == 0) return true;
    auto* d_bad = reinterpret_cast<uint32_t*>(s.d_bad.get());
    return xec_validate_blocks(s.data.get(), s.count * m_chunk_data_blocks, m_block_size, d_bad,
                               s.stream) == XEC_SUCCESS &&
           xec_hip::copy_to_host(h_bad, d_bad, sizeof(uint32_t), s.stream);
  });
  return ok && std::all_of(bad.begin(), bad.end(), [](uint32_t b) { return b == 0; });
}

// Each shard's device gets access to the root's memory where the pair allows
// it; a pair without peer access still exchanges (the runtime stages the
// copies) and is recorded as such, so the caller can tell peer DMA from a
// staged copy.  False only if a runtime call failed.
bool XorecBenchmarkHipMulti::enable_peers(int root) noexcept {
  bool ok = true;
  for (Shard& s : m_shards) {
    s.peer = xec_hip::enable_peer_access(s.device, root);
    ok = ok && s.peer != xec_hip::PeerAccess::kError;
  }
  return ok;
}

int XorecBenchmarkHipMulti::scatter_from(const uint8_t* d_root_data, int root) noexcept {
  if (d_root_data == nullptr || !enable_peers(root)) return -1;
  return each([&](const Shard& s) {
           return s.count == 0 ||
                  xec_hip::copy_peer(s.data.get(), s.device,
                                     d_root_data + s.first * m_chunk_data_size, root,
                                     s.count * m_chunk_data_size, s.stream);
         })
             ? 0
             : -1;
}

int XorecBenchmarkHipMulti::gather_parity_to(uint8_t* d_root_parity, int root) noexcept {
  if (d_root_parity == nullptr || !enable_peers(root)) return -1;
  return each([&](const Shard& s) {
           return s.count == 0 ||
                  xec_hip::copy_peer(d_root_parity + s.first * m_chunk_parity_size, root,
                                     s.parity.get(), s.device, s.count * m_chunk_parity_size,
                                     s.stream);
         })
             ? 0
             : -1;
}

bool XorecBenchmarkHipMulti::read_shard(size_t i, uint8_t* h_data, uint8_t* h_parity) const
    noexcept {
  if (i >= m_shards.size()) return false;
  const Shard& s = m_shards[i];
  if (s.count == 0) return true;
  const DeviceRestore restore;
  return xec_hip::set_device(s.device) &&
         xec_hip::copy_to_host(h_data, s.data.get(), s.count * m_chunk_data_size, s.stream) &&
         xec_hip::copy_to_host(h_parity, s.parity.get(), s.count * m_chunk_parity_size,
                               s.stream) &&
         xec_hip::synchronize(s.stream);
}

size_t XorecBenchmarkHipMulti::lost_data_blocks() const noexcept {
  size_t n = 0;
  const uint8_t* bm = m_block_bitmap.get();
  for (size_t c = 0; c < m_chunks; ++c)
    for (size_t i = 0; i < m_chunk_data_blocks; ++i) n += bm[c * m_chunk_tot_blocks + i] == 0;
  return n;
}
