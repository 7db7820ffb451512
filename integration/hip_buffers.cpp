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
  return hipHostMalloc(&p, bytes ? bytes : 64, hipHostMallocDefault) == hipSuccess
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

}  // namespace xec_hip
