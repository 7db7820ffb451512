// error_preserve.cpp -- the library and the caller's pending HIP error (GPU
// test program, built by tests/host/Makefile, run by
// tests/test_gpu_error_state.py).
//
//   error_preserve decode    xec_decode on a BUSY stream (the case where the
//                            library would query the stream and its events),
//                            bitmap-tile and work-list paths, with and without
//                            an error of the caller's pending: the decode is
//                            exact, and afterwards hipGetLastError() returns
//                            the caller's own error (or success if none)
//   error_preserve pipeline  the same around xec_pipeline_decode /
//                            xec_pipeline_encode over pageable host buffers
//   error_preserve inject    run with XEC_TEST_FAIL_LAUNCH=1: every library
//                            launch fails with hipErrorInvalidConfiguration;
//                            with the caller's error of THAT code pending,
//                            xec_encode / xec_decode / xec_erase must still
//                            report XEC_DEVICE_ERROR
// Prints "error_preserve <mode> ok" and exits 0 on success.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "xec.h"

namespace {

__global__ void spin(unsigned long long cycles) {
  const unsigned long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
}

__global__ void nop(int* p) {
  if (p) p[threadIdx.x] = 1;
}

// The caller's own invalid launch: 2048 threads per workgroup.
void caller_error() {
  nop<<<1, 2048>>>(nullptr);
}

int fails = 0;
void expect(bool ok, const std::string& what) {
  if (!ok) {
    std::printf("FAIL %s\n", what.c_str());
    ++fails;
  }
}

const char* nm(hipError_t e) { return hipGetErrorName(e); }

// One decode on a busy stream.  `sparse`: 1 stripe in 4 lost a block (the
// work-list path: staging + side upload); else every stripe (bitmap tiles).
void decode_case(bool pending, bool sparse) {
  const size_t S = 8192, k = 4, m = 1, bs = 256, row = k + m;
  const std::string tag = std::string(sparse ? "list" : "bitmap") + (pending ? " +pending" : "");
  uint8_t *d = nullptr, *p = nullptr, *dbm = nullptr;
  hipStream_t s = nullptr;
  expect(hipMalloc(&d, S * k * bs) == hipSuccess && hipMalloc(&p, S * m * bs) == hipSuccess &&
             hipMalloc(&dbm, S * row) == hipSuccess &&
             hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess,
         "alloc " + tag);
  expect(xec_fill_splitmix64(d, S, k * bs, 77, s) == XEC_SUCCESS &&
             xec_encode(d, p, S, bs, k, m, s) == XEC_SUCCESS && hipStreamSynchronize(s) == hipSuccess,
         "fill+encode " + tag);
  std::vector<uint8_t> want(S * k * bs), got(S * k * bs);
  expect(hipMemcpy(want.data(), d, want.size(), hipMemcpyDeviceToHost) == hipSuccess, "read " + tag);
  std::vector<uint8_t> bm(S * row, 1);
  for (size_t c = 0; c < S; ++c)
    if (!sparse || c % 4 == 1) bm[c * row + (c * 7) % k] = 0;
  uint8_t* hbm = nullptr;
  expect(hipHostMalloc(&hbm, bm.size(), hipHostMallocDefault) == hipSuccess, "pinned " + tag);
  std::memcpy(hbm, bm.data(), bm.size());
  expect(hipMemcpy(dbm, hbm, bm.size(), hipMemcpyHostToDevice) == hipSuccess &&
             xec_erase(d, p, S, bs, k, m, dbm, s) == XEC_SUCCESS &&
             hipStreamSynchronize(s) == hipSuccess,
         "erase " + tag);
  (void)hipGetLastError();
  spin<<<1, 64, 0, s>>>(100000000ull);  // ~50 ms: the stream is busy at the call
  if (pending) caller_error();
  const hipError_t before = hipPeekAtLastError();
  const xec_status st = xec_decode(d, p, S, bs, k, m, hbm, dbm, s);
  expect(st == XEC_SUCCESS, "decode status " + tag + ": " + std::to_string((int)st));
  const hipError_t after = hipGetLastError();
  expect(after == before, "pending error " + tag + ": " + nm(before) + " -> " + nm(after));
  expect(hipStreamSynchronize(s) == hipSuccess &&
             hipMemcpy(got.data(), d, got.size(), hipMemcpyDeviceToHost) == hipSuccess,
         "read back " + tag);
  expect(got == want, "decoded bytes " + tag);
  (void)hipHostFree(hbm);
  (void)hipFree(d);
  (void)hipFree(p);
  (void)hipFree(dbm);
  (void)hipStreamDestroy(s);
}

void pipeline_case(bool pending) {
  const size_t S = 64, k = 8, m = 2, bs = 4096, row = k + m;
  const std::string tag = pending ? "pipeline +pending" : "pipeline";
  std::vector<uint8_t> data(S * k * bs), parity(S * m * bs), want(S * m * bs);
  for (size_t i = 0; i < data.size(); ++i) data[i] = static_cast<uint8_t>(i * 2654435761u >> 13);
  for (size_t c = 0; c < S; ++c)
    for (size_t j = 0; j < m; ++j)
      for (size_t x = 0; x < bs; ++x) {
        uint8_t v = 0;
        for (size_t i = j; i < k; i += m) v ^= data[(c * k + i) * bs + x];
        want[(c * m + j) * bs + x] = v;
      }
  xec_pipeline* pl = nullptr;
  expect(xec_pipeline_create(&pl, 8, bs, k, m, 2) == XEC_SUCCESS, "create " + tag);
  if (pending) caller_error();
  hipError_t before = hipPeekAtLastError();
  expect(xec_pipeline_encode(pl, data.data(), parity.data(), S) == XEC_SUCCESS, "encode " + tag);
  hipError_t after = hipPeekAtLastError();
  expect(after == before, "pending error after encode " + tag + ": " + nm(before) + " -> " + nm(after));
  expect(parity == want, "parity " + tag);
  std::vector<uint8_t> bm(S * row, 1), lossy = data;
  for (size_t c = 0; c < S; ++c) {
    const size_t i = (c * 5) % k;
    bm[c * row + i] = 0;
    std::memset(lossy.data() + (c * k + i) * bs, 0, bs);
  }
  expect(xec_pipeline_decode(pl, lossy.data(), parity.data(), S, bm.data()) == XEC_SUCCESS,
         "decode " + tag);
  after = hipGetLastError();
  expect(after == before, "pending error after decode " + tag + ": " + nm(before) + " -> " + nm(after));
  expect(lossy == data, "decoded bytes " + tag);
  (void)xec_pipeline_destroy(pl);
}

void inject_case(bool pending) {
  const size_t S = 16, k = 4, m = 1, bs = 256;
  const std::string tag = pending ? "inject +pending" : "inject";
  uint8_t *d = nullptr, *p = nullptr, *dbm = nullptr;
  expect(hipMalloc(&d, S * k * bs) == hipSuccess && hipMalloc(&p, S * m * bs) == hipSuccess &&
             hipMalloc(&dbm, S * (k + m)) == hipSuccess,
         "alloc " + tag);
  std::vector<uint8_t> bm(S * (k + m), 1);
  bm[2] = 0;
  if (pending) caller_error();
  expect(hipPeekAtLastError() == (pending ? hipErrorInvalidConfiguration : hipSuccess),
         "the caller's error is InvalidConfiguration " + tag);
  expect(xec_encode(d, p, S, bs, k, m, nullptr) == XEC_DEVICE_ERROR, "encode reports " + tag);
  expect(xec_decode(d, p, S, bs, k, m, bm.data(), dbm, nullptr) == XEC_DEVICE_ERROR,
         "decode reports " + tag);
  expect(xec_erase(d, p, S, bs, k, m, dbm, nullptr) == XEC_DEVICE_ERROR, "erase reports " + tag);
  expect(hipGetLastError() == hipErrorInvalidConfiguration, "the launch failure is pending " + tag);
  (void)hipFree(d);
  (void)hipFree(p);
  (void)hipFree(dbm);
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "decode";
  if (xec_init(0) != XEC_SUCCESS) {
    std::printf("xec_init failed\n");
    return 2;
  }
  if (mode == "decode") {
    for (bool sparse : {false, true})
      for (bool pending : {false, true}) decode_case(pending, sparse);
  } else if (mode == "pipeline") {
    pipeline_case(false);
    pipeline_case(true);
  } else if (mode == "inject") {
    const char* e = std::getenv("XEC_TEST_FAIL_LAUNCH");
    if (e == nullptr || e[0] != '1') {
      std::printf("inject mode needs XEC_TEST_FAIL_LAUNCH=1\n");
      return 2;
    }
    inject_case(false);
    inject_case(true);
  } else {
    std::printf("unknown mode %s\n", mode.c_str());
    return 2;
  }
  if (fails == 0) std::printf("error_preserve %s ok\n", mode.c_str());
  std::fflush(stdout);
  std::_Exit(fails ? 1 : 0);
}
