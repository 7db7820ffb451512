// xec_validate.hip -- device-side validation payload and check.
//
// The reference's only correctness check is a per-block payload: random PCG
// bytes from offset 8, the block length (u32) at 4 and a rotate-add checksum
// (u32, crc = rotl(crc,3) + byte, seeded with the length) at 0
// (src/utils/utils.cpp:35-97), generated and validated on the host with a
// full device<->host copy each iteration (xorec_gpu_cmp_bm.cpp:25-37,91-104).
// Here both run where the data lives.  The checksum is a strictly sequential
// chain, so the unit of parallelism is the block: one lane owns one block and
// walks it with 16-byte accesses (generation: PCG32, utils.cpp:17-32, with
// state RANDOM_SEED + seed + block, stream 1; the wall-clock seed of the
// reference is replaced by an explicit one).
#include <hip/hip_runtime.h>
#include <cstdint>

#include "xec_kernels.h"

namespace xec {

namespace {

constexpr uint64_t kPcgMul = 6364136223846793005ull;
constexpr uint64_t kRandomSeed = 1896;  // RANDOM_SEED, utils.hpp:26

struct Pcg {
  uint64_t state, inc;
  __device__ uint32_t next() {
    const uint64_t old = state;
    state = old * kPcgMul + inc;
    const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    const uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((0u - rot) & 31u));
  }
  __device__ Pcg(uint64_t seed, uint64_t seq) : state(0), inc((seq << 1u) | 1u) {
    next();
    state += seed;
    next();
  }
};

__device__ __forceinline__ uint32_t rotl3(uint32_t x) { return (x << 3) | (x >> 29); }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void pattern_kernel(uint8_t* data, uint64_t nblocks, uint64_t bs,
                                                      uint64_t seed) {
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nblocks) return;
  uint8_t* blk = data + b * bs;
  Pcg rng(kRandomSeed + seed + b, 1);
  if (bs < 16) {
    const uint8_t v = (uint8_t)rng.next();
    for (uint64_t i = 0; i < bs; ++i) blk[i] = v;
    return;
  }
  uint32_t crc = (uint32_t)bs;
  uint64_t i = 8;
  if (bs % 16 == 0) {
    // bytes 8..15 first, then whole 16-byte granules
    uint32_t w[2] = {0, 0};
    for (int q = 0; q < 8; ++q) {
      const uint32_t v = rng.next() & 0xffu;
      w[q >> 2] |= v << (8 * (q & 3));
      crc = rotl3(crc) + v;
    }
    reinterpret_cast<uint32_t*>(blk)[2] = w[0];
    reinterpret_cast<uint32_t*>(blk)[3] = w[1];
    for (i = 16; i < bs; i += 16) {
      u32x4 g = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const uint32_t v = rng.next() & 0xffu;
        g[q >> 2] |= v << (8 * (q & 3));
        crc = rotl3(crc) + v;
      }
      *reinterpret_cast<u32x4*>(blk + i) = g;
    }
  } else {
    for (; i < bs; ++i) {
      const uint8_t v = (uint8_t)rng.next();
      blk[i] = v;
      crc = rotl3(crc) + v;
    }
  }
  const uint32_t len = (uint32_t)bs;
  for (int q = 0; q < 4; ++q) {
    blk[4 + q] = (uint8_t)(len >> (8 * q));
    blk[q] = (uint8_t)(crc >> (8 * q));
  }
}

__global__ __launch_bounds__(256) void validate_kernel(const uint8_t* data, uint64_t nblocks,
                                                       uint64_t bs, uint32_t* bad) {
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nblocks) return;
  const uint8_t* blk = data + b * bs;
  bool ok;
  if (bs < 2) {
    ok = false;
  } else if (bs < 16) {
    ok = true;
    for (uint64_t i = 1; i < bs; ++i) ok &= blk[i] == blk[0];
  } else {
    uint32_t len = 0, stored = 0;
    for (int q = 0; q < 4; ++q) {
      len |= (uint32_t)blk[4 + q] << (8 * q);
      stored |= (uint32_t)blk[q] << (8 * q);
    }
    uint32_t crc = (uint32_t)bs;
    uint64_t i = 8;
    if (bs % 16 == 0) {
      for (; i < 16; ++i) crc = rotl3(crc) + blk[i];
      for (; i < bs; i += 16) {
        const u32x4 g = *reinterpret_cast<const u32x4*>(blk + i);
#pragma unroll
        for (int q = 0; q < 16; ++q) crc = rotl3(crc) + ((g[q >> 2] >> (8 * (q & 3))) & 0xffu);
      }
    } else {
      for (; i < bs; ++i) crc = rotl3(crc) + blk[i];
    }
    ok = len == (uint32_t)bs && stored == crc;
  }
  if (!ok) atomicAdd(bad, 1u);
}

}  // namespace

hipError_t launch_pattern(void* d_data, uint64_t nblocks, uint64_t bs, uint64_t seed,
                          hipStream_t s) {
  if (nblocks == 0) return hipSuccess;
  pattern_kernel<<<(uint32_t)((nblocks + 255) / 256), 256, 0, s>>>(static_cast<uint8_t*>(d_data),
                                                                  nblocks, bs, seed);
  return hipGetLastError();
}

hipError_t launch_validate(const void* d_data, uint64_t nblocks, uint64_t bs, uint32_t* d_bad,
                           hipStream_t s) {
  if (hipMemsetAsync(d_bad, 0, sizeof(uint32_t), s) != hipSuccess) return hipErrorUnknown;
  if (nblocks == 0) return hipSuccess;
  validate_kernel<<<(uint32_t)((nblocks + 255) / 256), 256, 0, s>>>(
      static_cast<const uint8_t*>(d_data), nblocks, bs, d_bad);
  return hipGetLastError();
}

}  // namespace xec
