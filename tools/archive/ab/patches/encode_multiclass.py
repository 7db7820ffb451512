"""Candidate: multi-class encode tiles for short classes.  At k/m = 2, 4, 8 an
encode tile covers G = XEC_MC_LOADS/(k/m) consecutive parity classes of one
stripe over its 1 KiB column chunk (default 16 loads: G = 2 at 16+2, 4 at
16+4 / 32+8, 8 at 16+8), every one of the G*k/m member loads in flight before
the first XOR, G parity stores -- the 16+1 encode's load shape on the m > 1
shapes.  Needs m % G == 0; other shapes keep the class tile.

    XEC_MC_LOADS=16 tools/ab/build_variant.sh mc16 tools/ab/patches/encode_multiclass.py
"""
import os
import sys

p = sys.argv[1]
s = open(p).read()
loads = int(os.environ.get("XEC_MC_LOADS", "16"))

kernel = r'''
// ---------------------------------------------------------------------------
// encode, multi-class tiles (candidate): tile = (stripe c, class group q,
// chunk); classes q*G .. q*G+G-1, all G*NM loads in flight, G stores.
// ---------------------------------------------------------------------------
template <int NM, int G, bool NT, int T>
__global__ __launch_bounds__(T) void encode_mc_kernel(const uint8_t* __restrict__ data,
                                                      uint8_t* __restrict__ parity, Geometry g) {
  const uint64_t groups = g.m / G;
  for (uint64_t t0 = blockIdx.x; t0 < g.total_tiles; t0 += gridDim.x) {
    const uint64_t t = g.total_tiles - 1 - t0;
    const uint64_t chunk = t % g.tiles_per_block;
    const uint64_t cq = t / g.tiles_per_block;
    const uint64_t j0 = (cq % groups) * G, c = cq / groups;
    const uint64_t off = (chunk * (uint64_t)T + threadIdx.x) * 16;
    if (off >= g.bs) continue;
    const uint8_t* p = data + (c * g.k + j0) * g.bs + off;
    uint8_t* dst = parity + (c * g.m + j0) * g.bs;
    const uint64_t stride = g.m * g.bs;
    u32x4 v[NM][G];
#pragma unroll
    for (int r = 0; r < NM; ++r, p += stride) {
#pragma unroll
      for (int q = 0; q < G; ++q) v[r][q] = ld16<NT>(p + (uint64_t)q * g.bs);
    }
#pragma unroll
    for (int q = 0; q < G; ++q) {
      u32x4 acc = v[0][q];
#pragma unroll
      for (int r = 1; r < NM; ++r) acc ^= v[r][q];
      st16_block<NT, kEncodeStoreAux>(dst + (uint64_t)q * g.bs, off, acc);
    }
  }
}

// ---------------------------------------------------------------------------
// decode: every lost data block'''
anchor = '''
// ---------------------------------------------------------------------------
// decode: every lost data block'''
assert anchor in s
s = s.replace(anchor, kernel, 1)

old = '''template <int U, bool NT, int T>
hipError_t enc_nm(const void* d, void* p, const Geometry& g, uint32_t grid, uint32_t lds,
                  hipStream_t s) {
'''
new = '''template <int NM, bool NT, int T>
bool try_mc(const void* d, void* p, const Geometry& g0, uint32_t max_grid, uint32_t lds,
            hipStream_t s, hipError_t* err) {
  constexpr int G = %d / NM;
  if (G < 2 || g0.m %% G != 0) return false;
  Geometry g = g0;
  g.total_tiles = g.S * (g.m / G) * g.tiles_per_block;
  const uint32_t grid = grid_for(g.total_tiles, max_grid, T);
  encode_mc_kernel<NM, G, NT, T><<<grid, T, lds, s>>>(static_cast<const uint8_t*>(d),
                                                      static_cast<uint8_t*>(p), g);
  *err = hipGetLastError();
  return true;
}

template <int U, bool NT, int T>
hipError_t enc_nm(const void* d, void* p, const Geometry& g, uint32_t grid, uint32_t lds,
                  hipStream_t s) {
  if constexpr (U == 1) {
    hipError_t e = hipSuccess;
    const uint32_t mg = grid < g.total_tiles ? grid : 0u;
    if (g.nm == 2 && try_mc<2, NT, T>(d, p, g, mg, lds, s, &e)) return e;
    if (g.nm == 4 && try_mc<4, NT, T>(d, p, g, mg, lds, s, &e)) return e;
    if (g.nm == 8 && try_mc<8, NT, T>(d, p, g, mg, lds, s, &e)) return e;
  }
''' % loads
assert old in s
s = s.replace(old, new, 1)
open(p, "w").write(s)
