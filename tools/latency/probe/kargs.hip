#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int N> struct A { uint32_t n; uint32_t v[N]; };
template <int N> __global__ void k(A<N> a, uint32_t* out) { if (threadIdx.x == 0) out[0] = a.v[a.n % N]; }
template <int N> int run(uint32_t* d) {
  static A<N> a; a.n = N - 3; for (int i = 0; i < N; ++i) a.v[i] = i * 7 + 1;
  k<N><<<1, 64>>>(a, d);
  hipError_t e = hipGetLastError(); if (e != hipSuccess) { printf("N=%d launch error %s\n", N, hipGetErrorString(e)); return 1; }
  e = hipDeviceSynchronize(); if (e != hipSuccess) { printf("N=%d sync error %s\n", N, hipGetErrorString(e)); return 1; }
  uint32_t h = 0; hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  printf("N=%d bytes=%zu got %u want %u %s\n", N, sizeof(A<N>), h, (N - 3) * 7 + 1, h == (uint32_t)((N - 3) * 7 + 1) ? "OK" : "BAD");
  return 0;
}
int main() { uint32_t* d; hipMalloc(&d, 4); run<1000>(d); run<1900>(d); run<4000>(d); return 0; }
