// xorec_hip_bm.cpp -- see xorec_hip_bm.hpp.  Each method follows the
// XorecBenchmarkGpuCmp method it replaces (src/algorithms/xorec_gpu_cmp_bm.cpp)
// and uses the interface's utilities (utils.hpp) where that plugin does; the
// codec calls are include/xec.h.
#include "xorec_hip_bm.hpp"

#include <algorithm>
#include <cstdint>
#include <memory>

#include "hip_buffers.hpp"
#include "utils.hpp"

namespace {

using DevBuf = std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>>;

DevBuf device_buffer(size_t bytes) {
  uint8_t* p = xec_hip::alloc_device(bytes);
  if (p == nullptr) throw_error("XorecBenchmarkHip: hipMalloc failed");
  return DevBuf(p, xec_hip::free_device);
}

DevBuf pinned_buffer(size_t bytes) {
  uint8_t* p = xec_hip::alloc_pinned(bytes);
  if (p == nullptr) throw_error("XorecBenchmarkHip: hipHostMalloc failed");
  return DevBuf(p, xec_hip::free_pinned);
}

}  // namespace

XorecBenchmarkHip::XorecBenchmarkHip(const BenchmarkConfig& config)
  : XorecBenchmarkHip(config, XecPluginOptions{}) {}

// XorecBenchmarkGpuCmp ctor (xorec_gpu_cmp_bm.cpp:6-18): the base class's host
// buffers are replaced by device data / parity and a pinned host bitmap.  The
// reference's num_gpu_blocks / threads_per_gpu_block are not needed: the
// library picks the gfx950 launch shape.
XorecBenchmarkHip::XorecBenchmarkHip(const BenchmarkConfig& config,
                                     const XecPluginOptions& options)
  : AbstractBenchmark(config),
    m_opt(options),
    m_gpu_block_bitmap(nullptr, xec_hip::free_device),
    m_gpu_bad(nullptr, xec_hip::free_device),
    m_host_stage(nullptr, xec_hip::free_pinned) {
  if (!xec_hip::set_device(m_opt.device)) throw_error("XorecBenchmarkHip: bad device");
  (void)xec_hip::set_sync_mode(m_opt.sync_mode);  // before the context is active
  if (xec_init(m_opt.device) != XEC_SUCCESS) throw_error("XorecBenchmarkHip: xec_init failed");
  // Buffers first, the stream last: a constructor that throws runs no
  // destructor, so nothing it made may need one (the buffers free themselves
  // through their deleters).
  m_gpu_block_bitmap = device_buffer(m_chunks * m_chunk_tot_blocks);
  m_gpu_bad = device_buffer(sizeof(uint32_t));
  m_data_buf = device_buffer(m_chunks * m_chunk_data_size);
  m_parity_buf = device_buffer(m_chunks * m_chunk_parity_size);
  m_block_bitmap = pinned_buffer(m_chunks * m_chunk_tot_blocks);
  if (!m_opt.seeded || m_opt.host_check) m_host_stage = pinned_buffer(m_chunks * m_chunk_data_size);
  m_stream = xec_hip::create_stream();
  if (m_stream == nullptr) throw_error("XorecBenchmarkHip: hipStreamCreate failed");
}

XorecBenchmarkHip::~XorecBenchmarkHip() noexcept {
  (void)xec_hip::synchronize(m_stream);
  xec_hip::destroy_stream(m_stream);
}

// xorec_gpu_cmp_bm.cpp:20-23
void XorecBenchmarkHip::setup() noexcept {
  ++m_round;
  std::fill_n(m_block_bitmap.get(), m_chunks * m_chunk_tot_blocks, 1);
  m_write_data_buffer();
}

// xorec_gpu_cmp_bm.cpp:25-37: the reference's write_validation_pattern
// (utils.cpp:35-69) per block on the host, one copy to HBM.  Seeded: the same
// payload written on the device, block b of round r from seed + (r << 32) + b.
void XorecBenchmarkHip::m_write_data_buffer() noexcept {
  const size_t blocks = m_chunks * m_chunk_data_blocks;
  if (m_opt.seeded) {
    if (xec_write_validation_pattern(m_data_buf.get(), blocks, m_block_size,
                                     m_opt.seed + (m_round << 32), m_stream) != XEC_SUCCESS ||
        !xec_hip::synchronize(m_stream))
      throw_error("XorecBenchmarkHip: device payload failed");
    return;
  }
  uint8_t* stage = m_host_stage.get();
  const long long n = static_cast<long long>(blocks);
  bool failed = false;
#pragma omp parallel for schedule(static) reduction(|| : failed)
  for (long long b = 0; b < n; ++b)
    failed = write_validation_pattern(stage + static_cast<size_t>(b) * m_block_size,
                                      m_block_size) != 0 || failed;
  if (failed) throw_error("Failed to write random checking packet.");
  if (!xec_hip::copy_to_device(m_data_buf.get(), stage, m_chunks * m_chunk_data_size, m_stream) ||
      !xec_hip::synchronize(m_stream))
    throw_error("XorecBenchmarkHip: data upload failed");
}

// xorec_gpu_cmp_bm.cpp:39-52
int XorecBenchmarkHip::encode() noexcept {
  m_last_status = xec_encode(m_data_buf.get(), m_parity_buf.get(), m_chunks, m_block_size,
                             m_chunk_data_blocks, m_chunk_parity_blocks, m_stream);
  const bool synced = xec_hip::synchronize(m_stream);
  return (m_last_status == XEC_SUCCESS && synced) ? 0 : -1;
}

// xorec_gpu_cmp_bm.cpp:54-69.  The status is the reference's XorecResult
// numerically (include/xec.h); parity is read-only here.
int XorecBenchmarkHip::decode() noexcept {
  m_last_status = xec_decode(m_data_buf.get(), m_parity_buf.get(), m_chunks, m_block_size,
                             m_chunk_data_blocks, m_chunk_parity_blocks, m_block_bitmap.get(),
                             m_gpu_block_bitmap.get(), m_stream);
  const bool synced = xec_hip::synchronize(m_stream);
  return (static_cast<XorecResult>(m_last_status) == XorecResult::Success && synced) ? 0 : -1;
}

// xorec_gpu_cmp_bm.cpp:71-89: the reference's select_lost_blocks
// (utils.cpp:100-127) per stripe on the host bitmap (seeded: xec_select_lost_blocks,
// stripe c of round r from seed + (r << 32) + c), then one xec_erase kernel
// instead of one cudaMemset per lost block, synchronised so that no erasure
// work drains into decode's timer.
void XorecBenchmarkHip::simulate_data_loss() noexcept {
  uint8_t* bm = m_block_bitmap.get();
  for (size_t c = 0; c < m_chunks; ++c) {
    uint8_t* row = bm + c * m_chunk_tot_blocks;
    if (m_opt.seeded) {
      if (xec_select_lost_blocks(m_chunk_data_blocks, m_chunk_parity_blocks, m_chunk_lost_blocks,
                                 row, m_opt.seed + (m_round << 32) + c) != XEC_SUCCESS)
        throw_error("XorecBenchmarkHip: lost blocks must be <= parity blocks");
    } else {
      select_lost_blocks(m_chunk_data_blocks, m_chunk_parity_blocks, m_chunk_lost_blocks, row);
    }
  }
  if (!xec_hip::copy_to_device(m_gpu_block_bitmap.get(), bm, m_chunks * m_chunk_tot_blocks,
                               m_stream) ||
      xec_erase(m_data_buf.get(), m_parity_buf.get(), m_chunks, m_block_size,
                m_chunk_data_blocks, m_chunk_parity_blocks, m_gpu_block_bitmap.get(),
                m_stream) != XEC_SUCCESS ||
      !xec_hip::synchronize(m_stream))
    throw_error("XorecBenchmarkHip: erasure failed");
}

// xorec_gpu_cmp_bm.cpp:91-104: every data block's embedded checksum
// (validate_block, utils.cpp:72-97), checked on the device (xec_validate_blocks)
// instead of after a copy of the whole batch -- or, with host_check, after it.
bool XorecBenchmarkHip::check_for_corruption() const noexcept {
  const size_t blocks = m_chunks * m_chunk_data_blocks;
  if (m_opt.host_check) {
    uint8_t* stage = m_host_stage.get();
    if (!xec_hip::copy_to_host(stage, m_data_buf.get(), m_chunks * m_chunk_data_size, m_stream) ||
        !xec_hip::synchronize(m_stream))
      return false;
    const long long n = static_cast<long long>(blocks);
    long long bad = 0;
#pragma omp parallel for schedule(static) reduction(+ : bad)
    for (long long b = 0; b < n; ++b)
      bad += validate_block(stage + static_cast<size_t>(b) * m_block_size, m_block_size) ? 0 : 1;
    return bad == 0;
  }
  uint32_t bad = 1;
  auto* d_bad = reinterpret_cast<uint32_t*>(m_gpu_bad.get());
  if (xec_validate_blocks(m_data_buf.get(), blocks, m_block_size, d_bad, m_stream) !=
          XEC_SUCCESS ||
      !xec_hip::copy_to_host(&bad, d_bad, sizeof bad, m_stream) ||
      !xec_hip::synchronize(m_stream))
    return false;
  return bad == 0;
}

size_t XorecBenchmarkHip::lost_data_blocks() const noexcept {
  size_t n = 0;
  const uint8_t* bm = m_block_bitmap.get();
  for (size_t c = 0; c < m_chunks; ++c)
    for (size_t i = 0; i < m_chunk_data_blocks; ++i) n += bm[c * m_chunk_tot_blocks + i] == 0;
  return n;
}
