// last_error_probe.hip -- what HIP's per-thread "last error" holds after each
// kind of call the library makes while a caller's error is pending.  Decides
// how xec_api.cpp's stream_busy / event_passed / launch wrappers must behave
// to leave a caller's unread error in place.
//
//   make -C tools/lab last_error_probe && tools/lab/last_error_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void spin(unsigned long long cycles) {
  const unsigned long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
}

__global__ void nop(int* p) {
  if (p) p[threadIdx.x] = 1;
}

static const char* nm(hipError_t e) { return hipGetErrorName(e); }

static void bad_launch() {  // a caller's invalid launch: 2048 threads per block
  nop<<<1, 2048>>>(nullptr);
}

int main() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  int* d = nullptr;
  (void)hipMalloc(&d, 4096);
  (void)hipGetLastError();

  // 1. the caller's invalid launch: what is pending
  bad_launch();
  std::printf("1 after bad launch: peek=%s\n", nm(hipPeekAtLastError()));
  // 2. a successful API call while it is pending
  int dev = -1;
  (void)hipGetDevice(&dev);
  std::printf("2 after ok hipGetDevice: peek=%s\n", nm(hipPeekAtLastError()));
  // 3. a successful kernel launch (chevrons) while it is pending
  nop<<<1, 64, 0, s>>>(d);
  std::printf("3 after ok launch: peek=%s\n", nm(hipPeekAtLastError()));
  // 4. hipStreamQuery -> NotReady while it is pending
  spin<<<1, 64, 0, s>>>(200000000ull);
  const hipError_t q = hipStreamQuery(s);
  std::printf("4 hipStreamQuery busy -> %s, peek=%s\n", nm(q), nm(hipPeekAtLastError()));
  // 5. hipEventQuery -> NotReady while it is pending
  (void)hipEventRecord(ev, s);
  spin<<<1, 64, 0, s>>>(200000000ull);
  (void)hipEventRecord(ev, s);
  const hipError_t eq = hipEventQuery(ev);
  std::printf("5 hipEventQuery busy -> %s, peek=%s\n", nm(eq), nm(hipPeekAtLastError()));
  (void)hipStreamSynchronize(s);
  std::printf("5b after hipStreamSynchronize: peek=%s\n", nm(hipPeekAtLastError()));
  std::printf("5c get=%s then peek=%s\n", nm(hipGetLastError()), nm(hipPeekAtLastError()));

  // 6. clean thread: hipStreamQuery NotReady -> pending?
  spin<<<1, 64, 0, s>>>(200000000ull);
  const hipError_t q2 = hipStreamQuery(s);
  std::printf("6 clean: hipStreamQuery busy -> %s, peek=%s\n", nm(q2), nm(hipPeekAtLastError()));
  (void)hipGetLastError();
  (void)hipEventRecord(ev, s);
  const hipError_t eq2 = hipEventQuery(ev);
  std::printf("7 clean: hipEventQuery busy -> %s, peek=%s\n", nm(eq2), nm(hipPeekAtLastError()));
  (void)hipStreamSynchronize(s);
  (void)hipGetLastError();

  // 8. hipLaunchKernel's return value: a failing launch, clean and with an
  // error pending
  {
    int* p = nullptr;
    void* args[] = {&p};
    const hipError_t r = hipLaunchKernel(reinterpret_cast<const void*>(&nop), dim3(1), dim3(2048),
                                         args, 0, s);
    std::printf("8 clean: hipLaunchKernel bad -> %s, peek=%s\n", nm(r), nm(hipPeekAtLastError()));
    (void)hipGetLastError();
    bad_launch();
    const hipError_t r2 = hipLaunchKernel(reinterpret_cast<const void*>(&nop), dim3(1), dim3(64),
                                          args, 0, s);
    std::printf("9 pending: hipLaunchKernel ok -> %s, peek=%s\n", nm(r2),
                nm(hipPeekAtLastError()));
    const hipError_t r3 = hipLaunchKernel(reinterpret_cast<const void*>(&nop), dim3(1),
                                          dim3(4096), args, 0, s);
    std::printf("10 pending: hipLaunchKernel bad -> %s, peek=%s\n", nm(r3),
                nm(hipPeekAtLastError()));
    (void)hipGetLastError();
    // 11. pending error, then a failing hipMalloc (different code)
    bad_launch();
    void* huge = nullptr;
    const hipError_t r4 = hipMalloc(&huge, (size_t)1 << 50);
    std::printf("11 pending: hipMalloc huge -> %s, peek=%s\n", nm(r4), nm(hipPeekAtLastError()));
    (void)hipGetLastError();
    // 12. clean, hipStreamQuery idle
    (void)hipStreamSynchronize(s);
    const hipError_t q3 = hipStreamQuery(s);
    std::printf("12 clean idle: hipStreamQuery -> %s, peek=%s\n", nm(q3),
                nm(hipPeekAtLastError()));
  }
  (void)hipFree(d);
  return 0;
}
