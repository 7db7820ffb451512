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

}  // namespace

XorecBenchmarkHip::XorecBenchmarkHip(const BenchmarkConfig& config)
    : AbstractBenchmark(config), m_host_validation(config.host_validation), m_seed(config.seed) {
  if (xec_init(config.device_id) != XEC_SUCCESS) throw std::runtime_error("xec_init failed");
  if (config.sync_mode > 0) {
    static const unsigned flags[] = {0, hipDeviceScheduleSpin, hipDeviceScheduleYield,
                                     hipDeviceScheduleBlockingSync};
    // only possible before the device's context is active; ignored otherwise
    (void)hipSetDeviceFlags(flags[config.sync_mode & 3]);
  }
  check_hip(hipStreamCreateWithFlags(&m_stream, hipStreamNonBlocking), "hipStreamCreate");
  const size_t S = m_chunks;
  const size_t data_bytes = std::max<size_t>(S * m_chunk_data_size, 64);
  const size_t parity_bytes = std::max<size_t>(S * m_chunk_parity_size, 64);
  const size_t bitmap_bytes = std::max<size_t>(S * m_chunk_tot_blocks, 64);
  check_hip(hipMalloc(&m_data, data_bytes), "hipMalloc data");
  check_hip(hipMalloc(&m_parity, parity_bytes), "hipMalloc parity");
  check_hip(hipMalloc(&m_d_bitmap, bitmap_bytes), "hipMalloc bitmap");
  check_hip(hipMalloc(&m_d_erase, bitmap_bytes), "hipMalloc erase bitmap");
  check_hip(hipHostMalloc(&m_h_bitmap, bitmap_bytes, hipHostMallocDefault), "hipHostMalloc bitmap");
  check_hip(hipMalloc(&m_d_bad, sizeof(uint32_t)), "hipMalloc bad counter");
  if (m_host_validation)
    check_hip(hipHostMalloc(&m_h_stage, data_bytes, hipHostMallocDefault), "hipHostMalloc stage");
}

XorecBenchmarkHip::~XorecBenchmarkHip() noexcept {
  if (m_stream) (void)hipStreamSynchronize(m_stream);
  (void)hipFree(m_data);
  (void)hipFree(m_parity);
  (void)hipFree(m_d_bitmap);
  (void)hipFree(m_d_erase);
  (void)hipHostFree(m_h_bitmap);
  (void)hipFree(m_d_bad);
  if (m_h_stage) (void)hipHostFree(m_h_stage);
  if (m_stream) (void)hipStreamDestroy(m_stream);
}

// XorecBenchmarkGpuCmp::setup / m_write_data_buffer (xorec_gpu_cmp_bm.cpp:20-37):
// every block present, fresh validation payload generated on the host and
// copied into HBM.
void XorecBenchmarkHip::setup() noexcept {
  ++m_round;
  std::fill_n(m_h_bitmap, m_chunks * m_chunk_tot_blocks, uint8_t{1});
  write_data_buffer();
}

void XorecBenchmarkHip::write_data_buffer() noexcept {
  const long nblocks = static_cast<long>(m_chunks * m_chunk_data_blocks);
  const uint64_t base = m_seed + (m_round << 32);
  if (!m_host_validation) {
    (void)xec_write_validation_pattern(m_data, static_cast<size_t>(nblocks), m_block_size, base,
                                       m_stream);
    (void)hipStreamSynchronize(m_stream);
    return;
  }
  omp_set_num_threads(static_cast<int>(std::max<size_t>(m_threads, 1)));
#pragma omp parallel for schedule(static)
  for (long b = 0; b < nblocks; ++b)
    write_validation_block(m_h_stage + static_cast<size_t>(b) * m_block_size, m_block_size,
                           base + static_cast<uint64_t>(b));
  (void)hipMemcpyAsync(m_data, m_h_stage, m_chunks * m_chunk_data_size, hipMemcpyHostToDevice,
                       m_stream);
  (void)hipStreamSynchronize(m_stream);
}

// XorecBenchmarkGpuCmp::encode (xorec_gpu_cmp_bm.cpp:39-52)
int XorecBenchmarkHip::encode() noexcept {
  m_last_status = xec_encode(m_data, m_parity, m_chunks, m_block_size, m_chunk_data_blocks,
                             m_chunk_parity_blocks, m_stream);
  if (hipStreamSynchronize(m_stream) != hipSuccess) return -1;
  return m_last_status == XEC_SUCCESS ? 0 : -1;
}

// XorecBenchmarkGpuCmp::decode (xorec_gpu_cmp_bm.cpp:54-69)
int XorecBenchmarkHip::decode() noexcept {
  m_last_status = xec_decode(m_data, m_parity, m_chunks, m_block_size, m_chunk_data_blocks,
                             m_chunk_parity_blocks, m_h_bitmap, m_d_bitmap, m_stream);
  if (hipStreamSynchronize(m_stream) != hipSuccess) return -1;
  return m_last_status == XEC_SUCCESS ? 0 : -1;
}

// AbstractBenchmark::simulate_data_loss (abstract_bm.cpp:20-39): per stripe,
// select a recoverable erasure set and zero those blocks -- here with one
// device kernel, synchronised so no erasure work drains into decode's timer.
void XorecBenchmarkHip::simulate_data_loss() noexcept {
  const size_t tot = m_chunk_tot_blocks;
  for (size_t c = 0; c < m_chunks; ++c)
    select_lost_blocks(m_chunk_data_blocks, m_chunk_parity_blocks, m_chunk_lost_blocks,
                       m_h_bitmap + c * tot, m_seed + (m_round << 32) + c);
  (void)hipMemcpyAsync(m_d_erase, m_h_bitmap, m_chunks * tot, hipMemcpyHostToDevice, m_stream);
  (void)xec_erase(m_data, m_parity, m_chunks, m_block_size, m_chunk_data_blocks,
                  m_chunk_parity_blocks, m_d_erase, m_stream);
  (void)hipStreamSynchronize(m_stream);
}

// XorecBenchmarkGpuCmp::check_for_corruption (xorec_gpu_cmp_bm.cpp:91-104):
// copy the data back and validate every data block's embedded checksum.
bool XorecBenchmarkHip::check_for_corruption() const noexcept {
  if (!m_host_validation) {
    uint32_t bad = 1;
    if (xec_validate_blocks(m_data, m_chunks * m_chunk_data_blocks, m_block_size, m_d_bad,
                            m_stream) != XEC_SUCCESS ||
        hipMemcpyAsync(&bad, m_d_bad, sizeof bad, hipMemcpyDeviceToHost, m_stream) != hipSuccess ||
        hipStreamSynchronize(m_stream) != hipSuccess)
      return false;
    return bad == 0;
  }
  if (hipMemcpyAsync(m_h_stage, m_data, m_chunks * m_chunk_data_size, hipMemcpyDeviceToHost,
                     m_stream) != hipSuccess)
    return false;
  if (hipStreamSynchronize(m_stream) != hipSuccess) return false;
  const long nblocks = static_cast<long>(m_chunks * m_chunk_data_blocks);
  int bad = 0;
#pragma omp parallel for schedule(static) reduction(+ : bad)
  for (long b = 0; b < nblocks; ++b)
    bad += validate_block(m_h_stage + static_cast<size_t>(b) * m_block_size, m_block_size) ? 0 : 1;
  return bad == 0;
}

}  // namespace xec
