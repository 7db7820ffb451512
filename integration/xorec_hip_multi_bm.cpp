// xorec_hip_multi_bm.cpp -- see xorec_hip_multi_bm.hpp.  Each method follows
// the XorecBenchmarkGpuCmp method it replaces (src/algorithms/
// xorec_gpu_cmp_bm.cpp), per device range, with the reference's own utilities
// (src/utils/utils.hpp) where that plugin uses them; codec calls are
// include/xec.h.
#include "xorec_hip_multi_bm.hpp"

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <sstream>
#include <string>

#include "hip_buffers.hpp"
#include "utils.hpp"

namespace {

// The device list: XEC_DEVICES ("0,1,2,...", repeats allowed), else every
// visible device.  BenchmarkConfig carries no device field
// (bm_config.hpp:25-43), so the list travels beside it.
std::vector<int> plugin_devices() {
  std::vector<int> devs;
  const int visible = xec_hip::device_count();
  if (const char* env = std::getenv("XEC_DEVICES"); env != nullptr && *env != '\0') {
    std::stringstream ss(env);
    std::string tok;
    while (std::getline(ss, tok, ',')) {
      char* end = nullptr;
      const long d = std::strtol(tok.c_str(), &end, 10);
      if (tok.empty() || *end != '\0' || d < 0 || d >= visible)
        throw_error("XorecBenchmarkHipMulti: bad device '" + tok + "' in XEC_DEVICES");
      devs.push_back(static_cast<int>(d));
    }
  } else {
    for (int d = 0; d < visible; ++d) devs.push_back(d);
  }
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

// XorecBenchmarkGpuCmp ctor (xorec_gpu_cmp_bm.cpp:6-18), once per device range:
// the base class's host data / parity buffers are dropped (the batch lives in
// the devices' HBM) and the bitmap is pinned host memory every device reads.
XorecBenchmarkHipMulti::XorecBenchmarkHipMulti(const BenchmarkConfig& config)
  : AbstractBenchmark(config) {
  const DeviceRestore restore;
  const std::vector<int> devs = plugin_devices();
  m_data_buf = std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>>(nullptr, no_free);
  m_parity_buf = std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>>(nullptr, no_free);
  uint8_t* bm = xec_hip::alloc_pinned(m_chunks * m_chunk_tot_blocks);
  if (bm == nullptr) throw_error("XorecBenchmarkHipMulti: hipHostMalloc failed");
  m_block_bitmap = std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>>(bm, xec_hip::free_pinned);
  // contiguous ranges, the first m_chunks % n one stripe longer
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
      if (xec_init(s.device) != XEC_SUCCESS)  // also makes s.device current
        throw_error("XorecBenchmarkHipMulti: xec_init(" + std::to_string(s.device) + ") failed");
      s.stream = xec_hip::create_stream();
      if (s.stream == nullptr) throw_error("XorecBenchmarkHipMulti: hipStreamCreate failed");
      s.data = dev_buf(s.count * m_chunk_data_size);
      s.parity = dev_buf(s.count * m_chunk_parity_size);
      s.d_bitmap = dev_buf(s.count * m_chunk_tot_blocks);
      s.d_erase = dev_buf(s.count * m_chunk_tot_blocks);
      s.d_bad = dev_buf(sizeof(uint32_t));
    }
  } catch (...) {
    // no destructor runs for a throwing constructor: the streams made so far
    // go here, the buffers with m_shards
    for (Shard& s : m_shards)
      if (s.stream != nullptr && xec_hip::set_device(s.device)) xec_hip::destroy_stream(s.stream);
    throw;
  }
}

XorecBenchmarkHipMulti::~XorecBenchmarkHipMulti() noexcept {
  const DeviceRestore restore;
  for (Shard& s : m_shards) {
    if (s.stream == nullptr || !xec_hip::set_device(s.device)) continue;
    (void)xec_hip::synchronize(s.stream);
    xec_hip::destroy_stream(s.stream);
  }
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
  std::fill_n(m_block_bitmap.get(), m_chunks * m_chunk_tot_blocks, 1);
  m_write_data_buffer();
}

// xorec_gpu_cmp_bm.cpp:25-37 per device range: the reference's
// write_validation_pattern (utils.cpp:35-69) on the host, one copy per range.
void XorecBenchmarkHipMulti::m_write_data_buffer() noexcept {
  for (const Shard& s : m_shards) {
    if (s.count == 0) continue;
    auto staging = make_unique_aligned<uint8_t>(s.count * m_chunk_data_size);
    const long long blocks = static_cast<long long>(s.count * m_chunk_data_blocks);
    bool failed = false;
#pragma omp parallel for reduction(|| : failed)
    for (long long b = 0; b < blocks; ++b)
      failed = write_validation_pattern(&staging[b * m_block_size], m_block_size) != 0 || failed;
    if (failed) throw_error("Failed to write random checking packet.");
    const DeviceRestore restore;
    if (!xec_hip::set_device(s.device) ||
        !xec_hip::copy_to_device(s.data.get(), staging.get(), s.count * m_chunk_data_size,
                                 s.stream) ||
        !xec_hip::synchronize(s.stream))
      throw_error("XorecBenchmarkHipMulti: data upload failed");
  }
}

// xorec_gpu_cmp_bm.cpp:39-52, on every range at once
int XorecBenchmarkHipMulti::encode() noexcept {
  return each([&](const Shard& s) {
           return xec_encode(s.data.get(), s.parity.get(), s.count, m_block_size,
                             m_chunk_data_blocks, m_chunk_parity_blocks, s.stream) == XEC_SUCCESS;
         })
             ? 0
             : -1;
}

// xorec_gpu_cmp_bm.cpp:54-69.  All-or-nothing over the whole batch: every
// range is checked on the host first (is_recoverable per stripe,
// xorec_utils.hpp:160-175); only if all are recoverable does any device
// launch.  Parity is read-only (include/xec.h).
int XorecBenchmarkHipMulti::decode() noexcept {
  for (const Shard& s : m_shards) {
    int needs = 0;
    if (xec_check_bitmap(m_block_bitmap.get() + s.first * m_chunk_tot_blocks, s.count,
                         m_chunk_data_blocks, m_chunk_parity_blocks, &needs) != XEC_SUCCESS)
      return -1;
  }
  return each([&](const Shard& s) {
           return xec_decode(s.data.get(), s.parity.get(), s.count, m_block_size,
                             m_chunk_data_blocks, m_chunk_parity_blocks,
                             m_block_bitmap.get() + s.first * m_chunk_tot_blocks,
                             s.d_bitmap.get(), s.stream) == XEC_SUCCESS;
         })
             ? 0
             : -1;
}

// xorec_gpu_cmp_bm.cpp:71-89: the reference's select_lost_blocks
// (utils.cpp:100-127) per stripe on the host bitmap, then per range one
// xec_erase kernel instead of a cudaMemset per lost block.
void XorecBenchmarkHipMulti::simulate_data_loss() noexcept {
  for (size_t c = 0; c < m_chunks; ++c)
    select_lost_blocks(m_chunk_data_blocks, m_chunk_parity_blocks, m_chunk_lost_blocks,
                       m_block_bitmap.get() + c * m_chunk_tot_blocks);
  const bool ok = each([&](const Shard& s) {
    return xec_hip::copy_to_device(s.d_erase.get(),
                                   m_block_bitmap.get() + s.first * m_chunk_tot_blocks,
                                   s.count * m_chunk_tot_blocks, s.stream) &&
           xec_erase(s.data.get(), s.parity.get(), s.count, m_block_size, m_chunk_data_blocks,
                     m_chunk_parity_blocks, s.d_erase.get(), s.stream) == XEC_SUCCESS;
  });
  if (!ok) throw_error("XorecBenchmarkHipMulti: erasure failed");
}

// xorec_gpu_cmp_bm.cpp:91-104: every data block's embedded checksum
// (validate_block, utils.cpp:72-97), checked on its device.
bool XorecBenchmarkHipMulti::check_for_corruption() const noexcept {
  std::vector<uint32_t> bad(m_shards.size(), 1);
  size_t i = 0;
  const bool ok = each([&](const Shard& s) {
    auto* d_bad = reinterpret_cast<uint32_t*>(s.d_bad.get());
    return xec_validate_blocks(s.data.get(), s.count * m_chunk_data_blocks, m_block_size, d_bad,
                               s.stream) == XEC_SUCCESS &&
           xec_hip::copy_to_host(&bad[i++], d_bad, sizeof(uint32_t), s.stream);
  });
  return ok && std::all_of(bad.begin(), bad.end(), [](uint32_t b) { return b == 0; });
}

bool XorecBenchmarkHipMulti::enable_peers(int root) const noexcept {
  for (const Shard& s : m_shards)
    if (!xec_hip::enable_peer_access(s.device, root)) return false;
  return true;
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
