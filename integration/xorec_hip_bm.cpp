// xorec_hip_bm.cpp -- see xorec_hip_bm.hpp.  Each method follows the
// XorecBenchmarkGpuCmp method it replaces (src/algorithms/xorec_gpu_cmp_bm.cpp)
// and uses the reference's own utilities (src/utils/utils.hpp) where that
// plugin does; the codec calls are include/xec.h.
#include "xorec_hip_bm.hpp"

#include <algorithm>
#include <cstdint>
#include <memory>

#include "hip_buffers.hpp"
#include "utils.hpp"

namespace {

std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>> device_buffer(size_t bytes) {
  uint8_t* p = xec_hip::alloc_device(bytes);
  if (p == nullptr) throw_error("XorecBenchmarkHip: hipMalloc failed");
  return std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>>(p, xec_hip::free_device);
}

std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>> pinned_buffer(size_t bytes) {
  uint8_t* p = xec_hip::alloc_pinned(bytes);
  if (p == nullptr) throw_error("XorecBenchmarkHip: hipHostMalloc failed");
  return std::unique_ptr<uint8_t[], DeleterFunc<uint8_t>>(p, xec_hip::free_pinned);
}

}  // namespace

// XorecBenchmarkGpuCmp ctor (xorec_gpu_cmp_bm.cpp:6-18): the base class's host
// buffers are replaced by device data / parity and a pinned host bitmap.  The
// reference's num_gpu_blocks / threads_per_gpu_block are not needed: the
// library picks the gfx950 launch shape.
XorecBenchmarkHip::XorecBenchmarkHip(const BenchmarkConfig& config)
  : AbstractBenchmark(config),
    m_gpu_block_bitmap(device_buffer(m_chunks * m_chunk_tot_blocks)),
    m_gpu_bad(device_buffer(sizeof(uint32_t))) {
  if (xec_init(0) != XEC_SUCCESS) throw_error("XorecBenchmarkHip: xec_init(0) failed");
  m_stream = xec_hip::create_stream();
  if (m_stream == nullptr) throw_error("XorecBenchmarkHip: hipStreamCreate failed");
  m_data_buf = device_buffer(m_chunks * m_chunk_data_size);
  m_parity_buf = device_buffer(m_chunks * m_chunk_parity_size);
  m_block_bitmap = pinned_buffer(m_chunks * m_chunk_tot_blocks);
}

XorecBenchmarkHip::~XorecBenchmarkHip() noexcept {
  (void)xec_hip::synchronize(m_stream);
  xec_hip::destroy_stream(m_stream);
}

// xorec_gpu_cmp_bm.cpp:20-23
void XorecBenchmarkHip::setup() noexcept {
  std::fill_n(m_block_bitmap.get(), m_chunks * m_chunk_tot_blocks, 1);
  m_write_data_buffer();
}

// xorec_gpu_cmp_bm.cpp:25-37: the reference's write_validation_pattern
// (utils.cpp:35-69) on the host, one copy to HBM.
void XorecBenchmarkHip::m_write_data_buffer() noexcept {
  auto staging = make_unique_aligned<uint8_t>(m_chunks * m_chunk_data_size);
  for (size_t c = 0; c < m_chunks; ++c) {
    uint8_t* data_buf = staging.get() + c * m_chunk_data_size;
    for (size_t i = 0; i < m_chunk_data_blocks; ++i) {
      if (write_validation_pattern(&data_buf[i * m_block_size], m_block_size)) {
        throw_error("Failed to write random checking packet.");
      }
    }
  }
  if (!xec_hip::copy_to_device(m_data_buf.get(), staging.get(), m_chunks * m_chunk_data_size,
                               m_stream) ||
      !xec_hip::synchronize(m_stream))
    throw_error("XorecBenchmarkHip: data upload failed");
}

// xorec_gpu_cmp_bm.cpp:39-52
int XorecBenchmarkHip::encode() noexcept {
  const xec_status st = xec_encode(m_data_buf.get(), m_parity_buf.get(), m_chunks, m_block_size,
                                   m_chunk_data_blocks, m_chunk_parity_blocks, m_stream);
  const bool synced = xec_hip::synchronize(m_stream);
  return (st == XEC_SUCCESS && synced) ? 0 : -1;
}

// xorec_gpu_cmp_bm.cpp:54-69.  The status is the reference's XorecResult
// numerically (include/xec.h); parity is read-only here.
int XorecBenchmarkHip::decode() noexcept {
  const xec_status st = xec_decode(m_data_buf.get(), m_parity_buf.get(), m_chunks, m_block_size,
                                   m_chunk_data_blocks, m_chunk_parity_blocks,
                                   m_block_bitmap.get(), m_gpu_block_bitmap.get(), m_stream);
  const bool synced = xec_hip::synchronize(m_stream);
  return (static_cast<XorecResult>(st) == XorecResult::Success && synced) ? 0 : -1;
}

// xorec_gpu_cmp_bm.cpp:71-89: the reference's select_lost_blocks
// (utils.cpp:100-127) per stripe on the host bitmap, then one xec_erase kernel
// instead of one cudaMemset per lost block.
void XorecBenchmarkHip::simulate_data_loss() noexcept {
  for (size_t c = 0; c < m_chunks; ++c) {
    select_lost_blocks(m_chunk_data_blocks, m_chunk_parity_blocks, m_chunk_lost_blocks,
                       m_block_bitmap.get() + c * m_chunk_tot_blocks);
  }
  if (!xec_hip::copy_to_device(m_gpu_block_bitmap.get(), m_block_bitmap.get(),
                               m_chunks * m_chunk_tot_blocks, m_stream) ||
      xec_erase(m_data_buf.get(), m_parity_buf.get(), m_chunks, m_block_size,
                m_chunk_data_blocks, m_chunk_parity_blocks, m_gpu_block_bitmap.get(),
                m_stream) != XEC_SUCCESS ||
      !xec_hip::synchronize(m_stream))
    throw_error("XorecBenchmarkHip: erasure failed");
}

// xorec_gpu_cmp_bm.cpp:91-104: every data block's embedded checksum
// (validate_block, utils.cpp:72-97), checked on the device instead of after a
// D2H copy of the whole batch.
bool XorecBenchmarkHip::check_for_corruption() const noexcept {
  uint32_t bad = 1;
  auto* d_bad = reinterpret_cast<uint32_t*>(m_gpu_bad.get());
  if (xec_validate_blocks(m_data_buf.get(), m_chunks * m_chunk_data_blocks, m_block_size, d_bad,
                          m_stream) != XEC_SUCCESS ||
      !xec_hip::copy_to_host(&bad, d_bad, sizeof bad, m_stream) ||
      !xec_hip::synchronize(m_stream))
    return false;
  return bad == 0;
}
