// mix_kernels.hip -- what the HBM allows a single-erasure decode (NOT the product).
//
// Built into tools/lab/libmix.so by tools/lab/Makefile, driven by
// tools/lab/mix_ceiling.py.  Each kernel walks the product's work-list tiling
// (csrc/xec_kernels.hip decode_list_kernel: one-wave workgroups, tile = (list
// entry, 1 KiB chunk), tiles from the end of the batch, `nt` loads, `sc1`
// stores) over the same list, and does part of the decode's traffic:
//   MODE 0  reads only: the k/m - 1 surviving members + the class parity,
//           XOR-reduced; the result is stored only if it equals `magic` in all
//           four words, which random data never does (the loads stay live);
//   MODE 1  writes only: the rebuilt-block store, a value computed from the
//           address (no loads);
//   MODE 2  both: the product's decode, restated (fidelity check of the lab);
//   MODE 3  both, tiles walked entry-fastest (tile t -> entry t mod n, chunk
//           t / n): concurrent workgroups spread over many rebuilt blocks
//           instead of the product's few (destination order the other way round).
// So MODE 0 / MODE 1 time the decode's exact read and write streams on their
// own, and their sum is the time the two take one after the other.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const uint32_t __attribute__((address_space(4)))* const_u32_as4;

struct MixGeo {
  uint64_t k, m, bs, tiles_per_block, total_tiles;
};

__device__ __forceinline__ void store_sc1(uint8_t* block, uint64_t off, u32x4 v) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(block, 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, (uint32_t)off, 0, 16 /* sc1 */);
}

template <int NM, int MODE>
__global__ __launch_bounds__(64) void mix_kernel(uint8_t* data, const uint8_t* __restrict__ parity,
                                                 const uint32_t* __restrict__ items, MixGeo g,
                                                 uint32_t magic) {
  const uint64_t stride = g.m * g.bs;
  for (uint64_t t0 = blockIdx.x; t0 < g.total_tiles; t0 += gridDim.x) {
    const uint64_t t = g.total_tiles - 1 - t0;
    const uint64_t n = g.total_tiles / g.tiles_per_block;
    const uint64_t e = MODE == 3 ? t % n : t / g.tiles_per_block;
    const uint32_t item = *(const_u32_as4)(items + e);
    const uint64_t chunk = MODE == 3 ? t / n : t % g.tiles_per_block;
    const uint64_t c = item >> 8;
    const uint32_t i = item & 0xFFu;
    const uint32_t j = i % (uint32_t)g.m, r = i / (uint32_t)g.m;
    uint8_t* base = data + (c * g.k + j) * g.bs;
    uint8_t* dst = base + (uint64_t)r * stride;
    const uint64_t off = (chunk * 64 + threadIdx.x) * 16;
    if (off >= g.bs) continue;
    if constexpr (MODE == 1) {
      const u32x4 v = {(uint32_t)off ^ magic, (uint32_t)c, i, magic};
      store_sc1(dst, off, v);
      continue;
    } else {
      const uint8_t* sub = parity + (c * g.m + j) * g.bs + off;
      const uint8_t* p = base + off;
      u32x4 v[NM];
#pragma unroll
      for (int q = 0; q < NM; ++q, p += stride) {
        const uint8_t* src = q == (int)r ? sub : p;
        v[q] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src));
      }
      u32x4 acc = v[0];
#pragma unroll
      for (int q = 1; q < NM; ++q) acc ^= v[q];
      if constexpr (MODE == 0) {
        if (acc.x == magic && acc.y == magic && acc.z == magic && acc.w == magic)
          store_sc1(dst, off, acc);
      } else {
        store_sc1(dst, off, acc);
      }
    }
  }
}

template <int NM>
hipError_t launch_nm(int mode, uint8_t* d, const uint8_t* p, const uint32_t* items, MixGeo g,
                     uint32_t grid, uint32_t lds, hipStream_t s) {
  if (mode == 0) mix_kernel<NM, 0><<<grid, 64, lds, s>>>(d, p, items, g, 0x9E3779B9u);
  else if (mode == 1) mix_kernel<NM, 1><<<grid, 64, lds, s>>>(d, p, items, g, 0x9E3779B9u);
  else if (mode == 2) mix_kernel<NM, 2><<<grid, 64, lds, s>>>(d, p, items, g, 0x9E3779B9u);
  else mix_kernel<NM, 3><<<grid, 64, lds, s>>>(d, p, items, g, 0x9E3779B9u);
  return hipGetLastError();
}

}  // namespace

extern "C" int mix_launch(int mode, void* d_data, const void* d_parity, const uint32_t* d_items,
                          uint64_t n_items, uint64_t k, uint64_t m, uint64_t bs, uint32_t lds,
                          void* stream) {
  MixGeo g{k, m, bs, (bs + 1023) / 1024, 0};
  g.total_tiles = n_items * g.tiles_per_block;
  if (g.total_tiles == 0) return 0;
  const uint64_t cap = 0xFFFFFFFFull / 64;
  const uint32_t grid = (uint32_t)(g.total_tiles < cap ? g.total_tiles : cap);
  uint8_t* d = static_cast<uint8_t*>(d_data);
  const uint8_t* p = static_cast<const uint8_t*>(d_parity);
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e;
  switch (k / m) {
    case 1: e = launch_nm<1>(mode, d, p, d_items, g, grid, lds, s); break;
    case 2: e = launch_nm<2>(mode, d, p, d_items, g, grid, lds, s); break;
    case 4: e = launch_nm<4>(mode, d, p, d_items, g, grid, lds, s); break;
    case 8: e = launch_nm<8>(mode, d, p, d_items, g, grid, lds, s); break;
    case 16: e = launch_nm<16>(mode, d, p, d_items, g, grid, lds, s); break;
    case 32: e = launch_nm<32>(mode, d, p, d_items, g, grid, lds, s); break;
    default: return -2;
  }
  return e == hipSuccess ? 0 : -1;
}
