// xec_kernels.hip -- CDNA4 (gfx950) kernels of the XOR-EC hot path.
//
// Written for MI355X from the reference's *behaviour*
// (src/xorec/xorec.cpp:24-111: parity class i % m, single-erasure rebuild),
// not from its CUDA kernels: there are no atomics, no memset pass and no
// 8-byte grid-stride loop here (cf. xorec_gpu_cmp.cu:119-208).
//
// Work unit ("tile"): one parity class j of one stripe c over a contiguous
// column range of 256*U 16-byte granules.  A thread owns U granules of the
// column range and keeps every member of the class in flight at once:
//   encode: NM = k/m loads  (data blocks j, j+m, ...)      -> 1 parity store
//   decode: NM loads        (class members, lost one       -> 1 store into the
//                            replaced by the class parity)     lost data block
// so each wave-instruction is a fully coalesced 1 KiB global_load_dwordx4
// from one block and each lane has NM*U independent 16-byte loads in flight.
// The XOR reduction happens in registers; no LDS is needed because no byte is
// read twice and no cross-lane exchange is needed ("Why no LDS").
//
// All byte offsets are 64-bit: the batch may exceed 4 GiB (cf. the 32-bit
// indices of xorec_gpu_cmp.cu:127-131).
#include <hip/hip_runtime.h>
#include <cstdint>

#include "xec_kernels.h"

namespace xec {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

template <bool NT>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Decompose a tile index into (stripe c, class j, column chunk).
struct TileCoord {
  uint64_t c, j, chunk;
};

__device__ __forceinline__ TileCoord tile_coord(uint64_t t, const Geometry& g) {
  TileCoord tc;
  tc.chunk = t % g.tiles_per_block;
  uint64_t cj = t / g.tiles_per_block;
  tc.j = cj % g.m;
  tc.c = cj / g.m;
  return tc;
}

// XOR-reduce NM members (base + r*stride for r != subst, `sub` for r == subst)
// over this thread's U granules starting at granule offset g0, and store into
// dst.  `full` = every granule of the tile lies inside the block.
template <int NM, int U, bool NT>
__device__ __forceinline__ void reduce_store(const u32x4* base, uint64_t stride, const u32x4* sub,
                                             int subst, u32x4* dst, uint64_t g0, uint64_t gran,
                                             uint32_t nm_rt) {
  constexpr int kT = kThreads;
  if constexpr (NM > 0) {
    const u32x4* src[NM];
#pragma unroll
    for (int r = 0; r < NM; ++r) src[r] = (r == subst) ? sub : base + (uint64_t)r * stride;
    if (g0 + (uint64_t)(U - 1) * kT < gran) {
      u32x4 v[NM][U];
#pragma unroll
      for (int r = 0; r < NM; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) v[r][u] = ld16<NT>(src[r] + g0 + u * kT);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        u32x4 acc = v[0][u];
#pragma unroll
        for (int r = 1; r < NM; ++r) acc ^= v[r][u];
        st16<NT>(dst + g0 + u * kT, acc);
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        uint64_t gi = g0 + u * kT;
        if (gi < gran) {
          u32x4 acc = ld16<NT>(src[0] + gi);
#pragma unroll
          for (int r = 1; r < NM; ++r) acc ^= ld16<NT>(src[r] + gi);
          st16<NT>(dst + gi, acc);
        }
      }
    }
  } else {
    // Runtime member count: groups of 8 loads in flight per granule.
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint64_t gi = g0 + u * kT;
      if (gi >= gran) continue;
      u32x4 acc = {0u, 0u, 0u, 0u};
      uint32_t r = 0;
      for (; r + 8 <= nm_rt; r += 8) {
        u32x4 v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          int rr = (int)(r + q);
          const u32x4* s = (rr == subst) ? sub : base + (uint64_t)rr * stride;
          v[q] = ld16<NT>(s + gi);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) acc ^= v[q];
      }
      for (; r < nm_rt; ++r) {
        const u32x4* s = ((int)r == subst) ? sub : base + (uint64_t)r * stride;
        acc ^= ld16<NT>(s + gi);
      }
      st16<NT>(dst + gi, acc);
    }
  }
}

// ---------------------------------------------------------------------------
// encode: parity[c][j] = XOR_{r < k/m} data[c][j + r*m]      (xorec.cpp:37-57)
// ---------------------------------------------------------------------------
template <int NM, int U, bool NT>
__global__ __launch_bounds__(kThreads) void encode_kernel(const u32x4* __restrict__ data,
                                                          u32x4* __restrict__ parity, Geometry g) {
  for (uint64_t t = blockIdx.x; t < g.total_tiles; t += gridDim.x) {
    TileCoord tc = tile_coord(t, g);
    const u32x4* base = data + (tc.c * g.k + tc.j) * g.gran;
    u32x4* dst = parity + (tc.c * g.m + tc.j) * g.gran;
    uint64_t g0 = tc.chunk * (uint64_t)(kThreads * U) + threadIdx.x;
    reduce_store<NM, U, NT>(base, g.m * g.gran, nullptr, -1, dst, g0, g.gran, (uint32_t)g.nm);
  }
}

// ---------------------------------------------------------------------------
// decode: for the (at most one, checked on the host) lost data block L of
// class j: data[c][L] = parity[c][j] ^ XOR_{r != L} data[c][j + r*m]
//                                                            (xorec.cpp:79-108)
// The lost member is found with one byte load per lane and a wave ballot.
// ---------------------------------------------------------------------------
template <int NM, int U, bool NT>
__global__ __launch_bounds__(kThreads) void decode_kernel(u32x4* data,
                                                          const u32x4* __restrict__ parity,
                                                          const uint8_t* __restrict__ bitmap,
                                                          Geometry g) {
  const uint32_t nm = NM > 0 ? (uint32_t)NM : (uint32_t)g.nm;
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t t = blockIdx.x; t < g.total_tiles; t += gridDim.x) {
    TileCoord tc = tile_coord(t, g);
    const uint8_t* row = bitmap + tc.c * (g.k + g.m);
    int lost = -1;
    for (uint32_t b = 0; b < nm; b += 64) {
      uint32_t r = b + lane;
      bool z = (r < nm) && (row[tc.j + (uint64_t)r * g.m] == 0);
      uint64_t mask = __ballot(z);
      if (mask) {
        lost = (int)(b + (uint32_t)__builtin_ctzll(mask));
        break;
      }
    }
    lost = __builtin_amdgcn_readfirstlane(lost);
    if (lost < 0) continue;
    u32x4* base = data + (tc.c * g.k + tc.j) * g.gran;
    const uint64_t stride = g.m * g.gran;
    const u32x4* par = parity + (tc.c * g.m + tc.j) * g.gran;
    u32x4* dst = base + (uint64_t)lost * stride;
    uint64_t g0 = tc.chunk * (uint64_t)(kThreads * U) + threadIdx.x;
    reduce_store<NM, U, NT>(base, stride, par, lost, dst, g0, g.gran, nm);
  }
}

// ---------------------------------------------------------------------------
// erase: zero every block whose bitmap byte is 0 (abstract_bm.cpp:20-39)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void erase_kernel(u32x4* data, u32x4* parity,
                                                         const uint8_t* __restrict__ bitmap,
                                                         Geometry g) {
  const uint64_t tot = g.k + g.m;
  const uint64_t nblocks = g.S * tot;
  const u32x4 zero = {0u, 0u, 0u, 0u};
  for (uint64_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
    if (bitmap[b] != 0) continue;
    uint64_t c = b / tot, i = b % tot;
    u32x4* blk = i < g.k ? data + (c * g.k + i) * g.gran : parity + (c * g.m + (i - g.k)) * g.gran;
    for (uint64_t x = threadIdx.x; x < g.gran; x += kThreads) blk[x] = zero;
  }
}

// ---------------------------------------------------------------------------
// fill: splitmix64 stream per stripe, state seed_base + c
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix_at(uint64_t seed, uint64_t n) {
  uint64_t z = seed + (n + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kThreads) void fill_kernel(uint64_t* buf, uint64_t S, uint64_t words,
                                                        uint64_t seed_base) {
  for (uint64_t c = blockIdx.y; c < S; c += gridDim.y) {
    uint64_t* row = buf + c * words;
    const uint64_t seed = seed_base + c;
    for (uint64_t n = (uint64_t)blockIdx.x * kThreads + threadIdx.x; n < words;
         n += (uint64_t)gridDim.x * kThreads)
      row[n] = splitmix_at(seed, n);
  }
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
namespace {

template <int NM, int U, bool NT>
hipError_t launch_encode_t(const void* d, void* p, const Geometry& g, uint32_t grid,
                           hipStream_t s) {
  encode_kernel<NM, U, NT><<<grid, kThreads, 0, s>>>(static_cast<const u32x4*>(d),
                                                     static_cast<u32x4*>(p), g);
  return hipGetLastError();
}

template <int NM, int U, bool NT>
hipError_t launch_decode_t(void* d, const void* p, const uint8_t* bm, const Geometry& g,
                           uint32_t grid, hipStream_t s) {
  decode_kernel<NM, U, NT><<<grid, kThreads, 0, s>>>(static_cast<u32x4*>(d),
                                                     static_cast<const u32x4*>(p), bm, g);
  return hipGetLastError();
}

// Dispatch over the member count (k/m) the reference configs use
// (bm_config.cpp:7-11 and BASELINE.json: 1, 2, 4, 8, 16, 32), runtime otherwise.
#define XEC_NM_SWITCH(NMV, CALL)      \
  switch (NMV) {                      \
    case 1: { constexpr int NM = 1; CALL; } \
    case 2: { constexpr int NM = 2; CALL; } \
    case 4: { constexpr int NM = 4; CALL; } \
    case 8: { constexpr int NM = 8; CALL; } \
    case 16: { constexpr int NM = 16; CALL; } \
    case 32: { constexpr int NM = 32; CALL; } \
    default: { constexpr int NM = 0; CALL; } \
  }

template <bool NT>
hipError_t launch_encode_nt(const void* d, void* p, const Geometry& g, int unroll, uint32_t grid,
                            hipStream_t s) {
  if (unroll == 4) { XEC_NM_SWITCH(g.nm, return (launch_encode_t<NM, 4, NT>(d, p, g, grid, s))) }
  if (unroll == 2) { XEC_NM_SWITCH(g.nm, return (launch_encode_t<NM, 2, NT>(d, p, g, grid, s))) }
  XEC_NM_SWITCH(g.nm, return (launch_encode_t<NM, 1, NT>(d, p, g, grid, s)))
}

template <bool NT>
hipError_t launch_decode_nt(void* d, const void* p, const uint8_t* bm, const Geometry& g,
                            int unroll, uint32_t grid, hipStream_t s) {
  if (unroll == 4) { XEC_NM_SWITCH(g.nm, return (launch_decode_t<NM, 4, NT>(d, p, bm, g, grid, s))) }
  if (unroll == 2) { XEC_NM_SWITCH(g.nm, return (launch_decode_t<NM, 2, NT>(d, p, bm, g, grid, s))) }
  XEC_NM_SWITCH(g.nm, return (launch_decode_t<NM, 1, NT>(d, p, bm, g, grid, s)))
}

}  // namespace

hipError_t launch_encode(const void* d_data, void* d_parity, const Geometry& g,
                         const LaunchShape& ls, hipStream_t s) {
  uint32_t grid = grid_for(g.total_tiles, ls.max_grid);
  return ls.nt ? launch_encode_nt<true>(d_data, d_parity, g, ls.unroll, grid, s)
               : launch_encode_nt<false>(d_data, d_parity, g, ls.unroll, grid, s);
}

hipError_t launch_decode(void* d_data, const void* d_parity, const uint8_t* d_bitmap,
                         const Geometry& g, const LaunchShape& ls, hipStream_t s) {
  uint32_t grid = grid_for(g.total_tiles, ls.max_grid);
  return ls.nt ? launch_decode_nt<true>(d_data, d_parity, d_bitmap, g, ls.unroll, grid, s)
               : launch_decode_nt<false>(d_data, d_parity, d_bitmap, g, ls.unroll, grid, s);
}

hipError_t launch_erase(void* d_data, void* d_parity, const uint8_t* d_bitmap, const Geometry& g,
                        hipStream_t s) {
  uint64_t nblocks = g.S * (g.k + g.m);
  uint32_t grid = grid_for(nblocks, 65536);
  erase_kernel<<<grid, kThreads, 0, s>>>(static_cast<u32x4*>(d_data),
                                         static_cast<u32x4*>(d_parity), d_bitmap, g);
  return hipGetLastError();
}

hipError_t launch_fill(void* d_buf, uint64_t S, uint64_t words, uint64_t seed_base,
                       hipStream_t s) {
  uint64_t gx = (words + kThreads - 1) / kThreads;
  if (gx > 1024) gx = 1024;
  uint64_t gy = S < 65535 ? S : 65535;
  if (gx == 0 || gy == 0) return hipSuccess;
  fill_kernel<<<dim3((uint32_t)gx, (uint32_t)gy), kThreads, 0, s>>>(static_cast<uint64_t*>(d_buf),
                                                                   S, words, seed_base);
  return hipGetLastError();
}

}  // namespace xec
