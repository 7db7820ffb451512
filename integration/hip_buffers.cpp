// hip_buffers.cpp -- see hip_buffers.hpp.  HIP runtime only; no reference header.
#include "hip_buffers.hpp"

#include <hip/hip_runtime_api.h>

namespace xec_hip {

uint8_t* alloc_device(size_t bytes) {
  void* p = nullptr;
  return hipMalloc(&p, bytes ? bytes : 64) == hipSuccess ? static_cast<uint8_t*>(p) : nullptr;
}

uint8_t* alloc_pinned(size_t bytes) {
  void* p = nullptr;
  // portable: every device of the process may read it (XorecBenchmarkHipMulti)
  return hipHostMalloc(&p, bytes ? bytes : 64, hipHostMallocPortable) == hipSuccess
             ? static_cast<uint8_t*>(p)
             : nullptr;
}

void free_device(uint8_t* p) {
  if (p) (void)hipFree(p);
}

void free_pinned(uint8_t* p) {
  if (p) (void)hipHostFree(p);
}

bool copy_to_device(void* dst, const void* src, size_t bytes, hipStream_t stream) {
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream) == hipSuccess;
}

bool copy_to_host(void* dst, const void* src, size_t bytes, hipStream_t stream) {
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream) == hipSuccess;
}

bool synchronize(hipStream_t stream) { return hipStreamSynchronize(stream) == hipSuccess; }

hipStream_t create_stream() {
  hipStream_t s = nullptr;
  return hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess ? s : nullptr;
}

void destroy_stream(hipStream_t stream) {
  if (stream) (void)hipStreamDestroy(stream);
}

int device_count() {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

int current_device() {
  int d = -1;
  return hipGetDevice(&d) == hipSuccess ? d : -1;
}

bool set_device(int device) { return hipSetDevice(device) == hipSuccess; }

bool set_sync_mode(int mode) {
  static const unsigned flags[] = {0, hipDeviceScheduleSpin, hipDeviceScheduleYield,
                                   hipDeviceScheduleBlockingSync};
  if (mode <= 0 || mode > 3) return mode == 0;
  // only possible before the device's context is active: a later call is
  // refused by the runtime, and its error is this call's to clear
  if (hipSetDeviceFlags(flags[mode]) == hipSuccess) return true;
  (void)hipGetLastError();
  return false;
}

PeerAccess enable_peer_access(int device, int peer) {
  if (device == peer) return PeerAccess::kSameDevice;
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, device, peer) != hipSuccess) return PeerAccess::kError;
  if (!can) return PeerAccess::kStaged;  // copies still work: the runtime stages them
  const int prev = current_device();
  if (hipSetDevice(device) != hipSuccess) return PeerAccess::kError;
  const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();  // ours: clear it
  if (prev >= 0) (void)hipSetDevice(prev);
  return e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled ? PeerAccess::kEnabled
                                                                 : PeerAccess::kError;
}

bool copy_peer(void* dst, int dst_device, const void* src, int src_device, size_t bytes,
               hipStream_t stream) {
  return hipMemcpyPeerAsync(dst, dst_device, src, src_device, bytes, stream) == hipSuccess;
}

}  // namespace xec_hip
