// xorec_hip_bm.cpp -- see xorec_hip_bm.hpp.
#include "xorec_hip_bm.hpp"

#include <omp.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "ec_utils.hpp"
#include "xec.h"

namespace xec {

namespace {

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

void free_device(uint8_t* p) { (void)hipFree(p); }
void free_pinned(uint8_t* p) { (void)hipHostFree(p); }

Buffer device_buffer(size_t bytes, const char* what) {
  void* p = nullptr;
  check_hip(hipMalloc(&p, std::max<size_t>(bytes, 64)), what);
  return Buffer(static_cast<uint8_t*>(p), free_device);
}

Buffer pinned_buffer(size_t bytes, const char* what) {
  void* p = nullptr;
  check_hip(hipHostMalloc(&p, std::max<size_t>(bytes, 64), hipHostMallocDefault), what);
  return Buffer(static_cast<uint8_t*>(p), free_pinned);
}

}  // namespace

// XorecBenchmarkGpuCmp ctor (xorec_gpu_cmp_bm.cpp:6-18): the base class's host
// buffers are replaced by device data / parity and a pinned host bitmap.
XorecBenchmarkHip::XorecBenchmarkHip(const BenchmarkConfig& config)
    : AbstractBenchmark(config),
      m_d_bitmap(nullptr, free_device),
      m_d_erase(nullptr, free_device),
      m_h_stage(nullptr, free_pinned),
      m_d_bad(nullptr, free_device),
      m_host_validation(config.host_validation) {
  if (xec_init(config.device_id) != XEC_SUCCESS) throw std::runtime_error("xec_init failed");
  if (config.sync_mode > 0) {
    static const unsigned flags[] = {0, hipDeviceScheduleSpin, hipDeviceScheduleYield,
                                     hipDeviceScheduleBlockingSync};
    // only possible before the device's context is active; ignored otherwise
    (void)hipSetDeviceFlags(flags[config.sync_mode & 3]);
  }
  check_hip(hipStreamCreateWithFlags(&m_stream, hipStreamNonBlocking), "hipStreamCreate");
  const size_t S = m_chunks;
  const size_t data_bytes = S * m_chunk_data_size;
  const size_t bitmap_bytes = S * m_chunk_tot_blocks;
  m_data_buf = device_buffer(data_bytes, "hipMalloc data");
  m_parity_buf = device_buffer(S * m_chunk_parity_size, "hipMalloc parity");
  m_block_bitmap = pinned_buffer(bitmap_bytes, "hipHostMalloc bitmap");
  m_d_bitmap = device_buffer(bitmap_bytes, "hipMalloc bitmap");
  m_d_erase = device_buffer(bitmap_bytes, "hipMalloc erase bitmap");
  m_d_bad = device_buffer(sizeof(uint32_t), "hipMalloc bad counter");
  if (m_host_validation) m_h_stage = pinned_buffer(data_bytes, "hipHostMalloc stage");
}

XorecBenchmarkHip::~XorecBenchmarkHip() noexcept {
  if (m_stream) (void)hipStreamSynchronize(m_stream);
  // device / pinned buffers are released by their deleters after this body
  if (m_stream) (void)hipStreamDestroy(m_stream);
}

// XorecBenchmarkGpuCmp::setup (xorec_gpu_cmp_bm.cpp:20-23): every block
// present, fresh validation payload.
void XorecBenchmarkHip::setup() noexcept {
  ++m_round;
  std::fill_n(m_block_bitmap.get(), m_chunks * m_chunk_tot_blocks, uint8_t{1});
  m_write_data_buffer();
}

// XorecBenchmarkGpuCmp::m_write_data_buffer (xorec_gpu_cmp_bm.cpp:25-37):
// written on the device by default; with host_validation generated on the host
// and copied, as the reference does.
void XorecBenchmarkHip::m_write_data_buffer() noexcept {
  const long nblocks = static_cast<long>(m_chunks * m_chunk_data_blocks);
  if (!m_host_validation) {
    (void)xec_write_validation_pattern(m_data_buf.get(), static_cast<size_t>(nblocks),
                                       m_block_size, round_seed(0), m_stream);
    (void)hipStreamSynchronize(m_stream);
    return;
  }
  omp_set_num_threads(static_cast<int>(std::max<size_t>(m_threads, 1)));
#pragma omp parallel for schedule(static)
  for (long b = 0; b < nblocks; ++b)
    write_validation_block(m_h_stage.get() + static_cast<size_t>(b) * m_block_size, m_block_size,
                           round_seed(static_cast<uint64_t>(b)));
  (void)hipMemcpyAsync(m_data_buf.get(), m_h_stage.get(), m_chunks * m_chunk_data_size,
                       hipMemcpyHostToDevice, m_stream);
  (void)hipStreamSynchronize(m_stream);
}

// XorecBenchmarkGpuCmp::encode (xorec_gpu_cmp_bm.cpp:39-52)
int XorecBenchmarkHip::encode() noexcept {
  m_last_status = xec_encode(m_data_buf.get(), m_parity_buf.get(), m_chunks, m_block_size,
                             m_chunk_data_blocks, m_chunk_parity_blocks, m_stream);
  if (hipStreamSynchronize(m_stream) != hipSuccess) return -1;
  return m_last_status == XEC_SUCCESS ? 0 : -1;
}

// XorecBenchmarkGpuCmp::decode (xorec_gpu_cmp_bm.cpp:54-69)
int XorecBenchmarkHip::decode() noexcept {
  m_last_status = xec_decode(m_data_buf.get(), m_parity_buf.get(), m_chunks, m_block_size,
                             m_chunk_data_blocks, m_chunk_parity_blocks, m_block_bitmap.get(),
                             m_d_bitmap.get(), m_stream);
  if (hipStreamSynchronize(m_stream) != hipSuccess) return -1;
  return m_last_status == XEC_SUCCESS ? 0 : -1;
}

// AbstractBenchmark::simulate_data_loss (abstract_bm.cpp:20-39) on HBM: per
// stripe, select a recoverable erasure set on the host, then zero those blocks
// with one device kernel, synchronised so no erasure work drains into decode's
// timer (cf. the per-block cudaMemset of xorec_gpu_cmp_bm.cpp:71-89).
void XorecBenchmarkHip::simulate_data_loss() noexcept {
  const size_t tot = m_chunk_tot_blocks;
  uint8_t* bm = m_block_bitmap.get();
  for (size_t c = 0; c < m_chunks; ++c)
    select_lost_blocks(m_chunk_data_blocks, m_chunk_parity_blocks, m_chunk_lost_blocks,
                       bm + c * tot, round_seed(c));
  (void)hipMemcpyAsync(m_d_erase.get(), bm, m_chunks * tot, hipMemcpyHostToDevice, m_stream);
  (void)xec_erase(m_data_buf.get(), m_parity_buf.get(), m_chunks, m_block_size,
                  m_chunk_data_blocks, m_chunk_parity_blocks, m_d_erase.get(), m_stream);
  (void)hipStreamSynchronize(m_stream);
}

// XorecBenchmarkGpuCmp::check_for_corruption (xorec_gpu_cmp_bm.cpp:91-104):
// every data block's embedded checksum, on the device by default.
bool XorecBenchmarkHip::check_for_corruption() const noexcept {
  if (!m_host_validation) {
    uint32_t bad = 1;
    uint32_t* d_bad = reinterpret_cast<uint32_t*>(m_d_bad.get());
    if (xec_validate_blocks(m_data_buf.get(), m_chunks * m_chunk_data_blocks, m_block_size, d_bad,
                            m_stream) != XEC_SUCCESS ||
        hipMemcpyAsync(&bad, d_bad, sizeof bad, hipMemcpyDeviceToHost, m_stream) != hipSuccess ||
        hipStreamSynchronize(m_stream) != hipSuccess)
      return false;
    return bad == 0;
  }
  if (hipMemcpyAsync(m_h_stage.get(), m_data_buf.get(), m_chunks * m_chunk_data_size,
                     hipMemcpyDeviceToHost, m_stream) != hipSuccess)
    return false;
  if (hipStreamSynchronize(m_stream) != hipSuccess) return false;
  const long nblocks = static_cast<long>(m_chunks * m_chunk_data_blocks);
  int bad = 0;
#pragma omp parallel for schedule(static) reduction(+ : bad)
  for (long b = 0; b < nblocks; ++b)
    bad += validate_block(m_h_stage.get() + static_cast<size_t>(b) * m_block_size, m_block_size)
               ? 0
               : 1;
  return bad == 0;
}

}  // namespace xec
