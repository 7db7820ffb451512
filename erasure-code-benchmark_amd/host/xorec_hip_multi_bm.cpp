// xorec_hip_multi_bm.cpp -- see xorec_hip_multi_bm.hpp.
#include "xorec_hip_multi_bm.hpp"

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

// The current device on entry is restored on exit.
struct DeviceRestore {
  int dev = 0;
  DeviceRestore() { (void)hipGetDevice(&dev); }
  ~DeviceRestore() { (void)hipSetDevice(dev); }
};

}  // namespace

XorecBenchmarkHipMulti::XorecBenchmarkHipMulti(const BenchmarkConfig& config)
    : AbstractBenchmark(config) {
  const DeviceRestore restore;
  std::vector<int> devs = config.devices;
  if (devs.empty()) {
    int n = 0;
    check_hip(hipGetDeviceCount(&n), "hipGetDeviceCount");
    for (int d = 0; d < n; ++d) devs.push_back(d);
  }
  if (devs.empty()) throw std::runtime_error("no HIP device");
  // the host copies of the base class are not used: the batch lives in the
  // devices' HBM, the bitmap in pinned host memory every device can read
  m_data_buf = Buffer(nullptr, free_device);
  m_parity_buf = Buffer(nullptr, free_device);
  void* bm = nullptr;
  check_hip(hipHostMalloc(&bm, std::max<size_t>(m_chunks * m_chunk_tot_blocks, 64),
                          hipHostMallocPortable),
            "hipHostMalloc bitmap");
  m_block_bitmap = Buffer(static_cast<uint8_t*>(bm), free_pinned);
  // contiguous stripe ranges, the first S % n shards one stripe longer
  // (xec.partition.stripe_range)
  const size_t n = devs.size(), base = m_chunks / n, extra = m_chunks % n;
  m_shards.resize(n);
  try {
    for (size_t i = 0; i < n; ++i) {
      Shard& s = m_shards[i];
      s.device = devs[i];
      s.first = i * base + std::min(i, extra);
      s.count = base + (i < extra ? 1 : 0);
      if (xec_init(s.device) != XEC_SUCCESS)
        throw std::runtime_error("xec_init(" + std::to_string(s.device) + ") failed");
      check_hip(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking), "hipStreamCreate");
      s.data = device_buffer(s.count * m_chunk_data_size, "hipMalloc data");
      s.parity = device_buffer(s.count * m_chunk_parity_size, "hipMalloc parity");
      s.d_bitmap = device_buffer(s.count * m_chunk_tot_blocks, "hipMalloc bitmap");
      s.d_erase = device_buffer(s.count * m_chunk_tot_blocks, "hipMalloc erase bitmap");
      s.d_bad = device_buffer(sizeof(uint32_t), "hipMalloc bad counter");
    }
    m_pool = std::make_unique<ShardPool>(n);
  } catch (...) {
    // a throwing constructor runs no destructor: release the streams made so
    // far here (the buffers go with m_shards)
    destroy_streams();
    throw;
  }
}

void XorecBenchmarkHipMulti::destroy_streams() noexcept {
  for (Shard& s : m_shards) {
    if (s.stream == nullptr) continue;
    (void)hipSetDevice(s.device);
    (void)hipStreamSynchronize(s.stream);
    (void)hipStreamDestroy(s.stream);
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
    ok &= hipSetDevice(s.device) == hipSuccess && fn(s);
  for (const Shard& s : m_shards)  // ... then wait for every device
    ok &= hipSetDevice(s.device) == hipSuccess && hipStreamSynchronize(s.stream) == hipSuccess;
  return ok;
}

// XorecBenchmarkGpuCmp::setup (xorec_gpu_cmp_bm.cpp:20-23)
void XorecBenchmarkHipMulti::setup() noexcept {
  ++m_round;
  std::fill_n(m_block_bitmap.get(), m_chunks * m_chunk_tot_blocks, uint8_t{1});
  m_write_data_buffer();
}

// Payload of global data block b seeded round_seed(b), on the devices.
void XorecBenchmarkHipMulti::m_write_data_buffer() noexcept {
  (void)each([&](const Shard& s) {
    return xec_write_validation_pattern(s.data.get(), s.count * m_chunk_data_blocks,
                                        m_block_size, round_seed(s.first * m_chunk_data_blocks),
                                        s.stream) == XEC_SUCCESS;
  });
}

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

// All-or-nothing over the WHOLE batch, like the one-device plugin and the
// reference's GPU decode (xorec_gpu_cmp.cu:75-81): each shard's thread (m_pool)
// first checks its slice of the host bitmap (xec_check_bitmap, is_recoverable
// per stripe, xorec_utils.hpp:160-175), then all meet (Rendezvous); if any
// stripe of any shard is unrecoverable no shard launches anything and the
// call returns DecodeFailure, so the bytes after a failed decode do not depend
// on the device count.  Otherwise every shard decodes its slice (xec_decode:
// host scan, then the launch) on its own thread, so no device's launch waits
// for another's scan; then every stream is waited for.
// The library's tuning overrides are per thread (include/xec.h): the caller's
// are copied into every worker before its xec_decode, so all shards launch the
// shape the caller configured, not the workers' defaults.
int XorecBenchmarkHipMulti::decode() noexcept {
  const size_t n = m_shards.size();
  std::vector<int> st(n, XEC_DEVICE_ERROR);
  Rendezvous all_recoverable(n);
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
    const int check = xec_check_bitmap(bm, s.count, m_chunk_data_blocks, m_chunk_parity_blocks,
                                       &needs);
    const bool go = all_recoverable.arrive(check == XEC_SUCCESS);
    if (i == 0) launched = go;
    if (!go) {
      st[i] = check;  // this shard's own verdict (0 if only another shard failed)
      return;
    }
    const DeviceRestore restore;
    if (hipSetDevice(s.device) != hipSuccess) return;
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
  return ok && status == XEC_SUCCESS ? 0 : -1;
}

// AbstractBenchmark::simulate_data_loss (abstract_bm.cpp:20-39): erasure sets
// drawn per GLOBAL stripe on the host, zeroed on each device by one kernel.
void XorecBenchmarkHipMulti::simulate_data_loss() noexcept {
  const size_t tot = m_chunk_tot_blocks;
  uint8_t* bm = m_block_bitmap.get();
  for (size_t c = 0; c < m_chunks; ++c)
    select_lost_blocks(m_chunk_data_blocks, m_chunk_parity_blocks, m_chunk_lost_blocks,
                       bm + c * tot, round_seed(c));
  (void)each([&](const Shard& s) {
    return hipMemcpyAsync(s.d_erase.get(), bm + s.first * tot, s.count * tot,
                          hipMemcpyHostToDevice, s.stream) == hipSuccess &&
           xec_erase(s.data.get(), s.parity.get(), s.count, m_block_size, m_chunk_data_blocks,
                     m_chunk_parity_blocks, s.d_erase.get(), s.stream) == XEC_SUCCESS;
  });
}

// XorecBenchmarkGpuCmp::check_for_corruption (xorec_gpu_cmp_bm.cpp:91-104):
// every data block's embedded checksum, on its device.
bool XorecBenchmarkHipMulti::check_for_corruption() const noexcept {
  std::vector<uint32_t> bad(m_shards.size(), 1);
  size_t i = 0;
  const bool ok = each([&](const Shard& s) {
    uint32_t* d_bad = reinterpret_cast<uint32_t*>(s.d_bad.get());
    uint32_t* h_bad = &bad[i++];
    return xec_validate_blocks(s.data.get(), s.count * m_chunk_data_blocks, m_block_size, d_bad,
                               s.stream) == XEC_SUCCESS &&
           hipMemcpyAsync(h_bad, d_bad, sizeof(uint32_t), hipMemcpyDeviceToHost, s.stream) ==
               hipSuccess;
  });
  return ok && std::all_of(bad.begin(), bad.end(), [](uint32_t b) { return b == 0; });
}

// Every shard device reads (scatter) or writes (gather) root's HBM: give it
// peer access to root where the pair supports it (otherwise the runtime
// stages the copy).  An access already enabled is fine.
bool XorecBenchmarkHipMulti::enable_peer(int root) noexcept {
  const DeviceRestore restore;
  for (const Shard& s : m_shards) {
    if (s.device == root) continue;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, s.device, root) != hipSuccess) return false;
    if (!can) continue;
    if (hipSetDevice(s.device) != hipSuccess) return false;
    const hipError_t e = hipDeviceEnablePeerAccess(root, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return false;
    (void)hipGetLastError();  // clear a sticky "already enabled"
  }
  return true;
}

int XorecBenchmarkHipMulti::scatter_from(const uint8_t* d_root_data, int root) noexcept {
  if (d_root_data == nullptr || !enable_peer(root)) return -1;
  const bool ok = each([&](const Shard& s) {
    return s.count == 0 ||
           hipMemcpyPeerAsync(s.data.get(), s.device, d_root_data + s.first * m_chunk_data_size,
                              root, s.count * m_chunk_data_size, s.stream) == hipSuccess;
  });
  return ok ? 0 : -1;
}

int XorecBenchmarkHipMulti::gather_parity_to(uint8_t* d_root_parity, int root) noexcept {
  if (d_root_parity == nullptr || !enable_peer(root)) return -1;
  const bool ok = each([&](const Shard& s) {
    return s.count == 0 ||
           hipMemcpyPeerAsync(d_root_parity + s.first * m_chunk_parity_size, root,
                              s.parity.get(), s.device, s.count * m_chunk_parity_size,
                              s.stream) == hipSuccess;
  });
  return ok ? 0 : -1;
}

bool XorecBenchmarkHipMulti::read_shard(size_t i, uint8_t* h_data, uint8_t* h_parity) const
    noexcept {
  if (i >= m_shards.size()) return false;
  const DeviceRestore restore;
  const Shard& s = m_shards[i];
  return hipSetDevice(s.device) == hipSuccess &&
         hipMemcpyAsync(h_data, s.data.get(), s.count * m_chunk_data_size, hipMemcpyDeviceToHost,
                        s.stream) == hipSuccess &&
         hipMemcpyAsync(h_parity, s.parity.get(), s.count * m_chunk_parity_size,
                        hipMemcpyDeviceToHost, s.stream) == hipSuccess &&
         hipStreamSynchronize(s.stream) == hipSuccess;
}

}  // namespace xec
