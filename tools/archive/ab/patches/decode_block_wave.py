"""Candidate: config 4's decode with one wave per 4 KiB block (stripe tiles).
The product's stripe tile is (stripe, 1 KiB chunk): a 4 KiB rebuilt block is
written as four 1 KiB pieces by four workgroups on four XCDs.  Here one wave
owns the stripe: lane granules lane*16 + u*1 KiB (u < 4), members taken G at a
time with all G*4 loads in flight, four accumulators, then the block leaves as
four 1 KiB wave-stores from one wave (write-only streams: 4.8 TB/s with 1 KiB
per workgroup, 6.5-7.0 with 4 KiB).  XEC_BW_G at patch time
(members per group, default 8); XEC_BW_ENC=1 also gives encode the shape.

    XEC_BW_G=8 tools/ab/build_variant.sh bw8 tools/ab/patches/decode_block_wave.py
"""
import os
import sys

p = sys.argv[1]
s = open(p).read()
G = int(os.environ.get("XEC_BW_G", "8"))
enc = os.environ.get("XEC_BW_ENC", "0") == "1"

kernel = r'''
// ---------------------------------------------------------------------------
// candidate: one wave per 4 KiB block (decode_block_wave.py)
// ---------------------------------------------------------------------------
template <int NM, int G>
__device__ __forceinline__ void xor_block4k(const uint8_t* base, uint64_t stride, const uint8_t* sub,
                                            int subst, uint8_t* dst, int aux_decode) {
  const uint64_t off = (uint64_t)threadIdx.x * 16;
  u32x4 acc[4] = {};
#pragma unroll
  for (int r0 = 0; r0 < NM; r0 += G) {
    u32x4 v[G][4];
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int r = r0 + q;
      const uint8_t* src = (r == subst ? sub : base + (uint64_t)r * stride) + off;
#pragma unroll
      for (int u = 0; u < 4; ++u) v[q][u] = ld16<true>(src + u * 1024);
    }
#pragma unroll
    for (int q = 0; q < G; ++q)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] ^= v[q][u];
  }
  if (aux_decode) {
#pragma unroll
    for (int u = 0; u < 4; ++u) st16_block<true, kDecodeStoreAux>(dst, off + u * 1024, acc[u]);
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) st16_block<true, kEncodeStoreAux>(dst, off + u * 1024, acc[u]);
  }
}

template <int NM, int G>
__global__ __launch_bounds__(64) void decode_block4k_kernel(uint8_t* data,
                                                            const uint8_t* __restrict__ parity,
                                                            const uint8_t* __restrict__ bitmap,
                                                            Geometry g) {
  if (g.gate != nullptr && *(const_i32_as4)g.gate != 0) return;
  const uint32_t m = (uint32_t)g.m;
  const uint64_t stride = g.m * g.bs;
  for (uint64_t t0 = blockIdx.x; t0 < g.S; t0 += gridDim.x) {
    const uint64_t c = g.S - 1 - t0;
    const uint64_t rowaddr = reinterpret_cast<uint64_t>(bitmap + c * (g.k + g.m));
    const uint64_t end = rowaddr + g.k;
    uint8_t* sdata = data + c * g.k * g.bs;
    const uint8_t* spar = parity + c * g.m * g.bs;
    for (uint64_t a = rowaddr & ~3ull; a < end; a += 4) {
      const uint32_t w = *(const_u32_as4)a;
      uint32_t z = ~(((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w) & 0x80808080u;
      if (a < rowaddr) z &= 0xFFFFFFFFu << (8 * (uint32_t)(rowaddr - a));
      if (a + 4 > end) z &= 0xFFFFFFFFu >> (8 * (uint32_t)(a + 4 - end));
      while (z) {
        const uint32_t i = (uint32_t)(a - rowaddr) + ((uint32_t)__builtin_ctz(z) >> 3);
        z &= z - 1;
        const uint32_t j = i % m, r = i / m;
        uint8_t* base = sdata + (uint64_t)j * g.bs;
        xor_block4k<NM, G>(base, stride, spar + (uint64_t)j * g.bs, (int)r,
                           base + (uint64_t)r * stride, 1);
      }
    }
  }
}

template <int NM, int G>
__global__ __launch_bounds__(64) void encode_block4k_kernel(const uint8_t* __restrict__ data,
                                                            uint8_t* __restrict__ parity,
                                                            Geometry g) {
  const uint64_t n = g.S * g.m;
  for (uint64_t t0 = blockIdx.x; t0 < n; t0 += gridDim.x) {
    const uint64_t cj = n - 1 - t0;
    const uint64_t j = cj % g.m, c = cj / g.m;
    xor_block4k<NM, G>(data + (c * g.k + j) * g.bs, g.m * g.bs, nullptr, -1,
                       parity + (c * g.m + j) * g.bs, 0);
  }
}

// ---------------------------------------------------------------------------
// host-side launchers'''
anchor = '''
// ---------------------------------------------------------------------------
// host-side launchers'''
assert anchor in s
s = s.replace(anchor, kernel, 1)

old = '''  if (tiling == kDecodeStripeTiles) g.total_tiles = g.S * g.tiles_per_block;'''
new = '''  if (tiling == kDecodeStripeTiles) g.total_tiles = g.S * g.tiles_per_block;
  if (tiling == kDecodeStripeTiles && g.bs == 4096 && g.nm == 32 && ls.threads == 64 &&
      ls.unroll == 1 && ls.nt && g.S > 0) {
    const uint32_t grid = grid_for(g.S, ls.max_grid, 64);
    decode_block4k_kernel<32, %d><<<grid, 64, ls.lds_bytes, s>>>(
        static_cast<uint8_t*>(d_data), static_cast<const uint8_t*>(d_parity), d_bitmap, g);
    return hipGetLastError();
  }''' % G
assert old in s
s = s.replace(old, new, 1)

if enc:
    old = '''  const uint32_t grid = grid_for(g.total_tiles, ls.max_grid, ls.threads);
  const uint32_t lds = ls.lds_bytes;
  if (ls.threads == 256)
    return ls.nt ? enc_u'''
    new = '''  if (g.bs == 4096 && g.nm == 32 && ls.threads == 64 && ls.unroll == 1 && ls.nt && g.S > 0) {
    const uint32_t grid = grid_for(g.S * g.m, ls.max_grid, 64);
    encode_block4k_kernel<32, %d><<<grid, 64, ls.lds_bytes, s>>>(
        static_cast<const uint8_t*>(d_data), static_cast<uint8_t*>(d_parity), g);
    return hipGetLastError();
  }
  const uint32_t grid = grid_for(g.total_tiles, ls.max_grid, ls.threads);
  const uint32_t lds = ls.lds_bytes;
  if (ls.threads == 256)
    return ls.nt ? enc_u''' % G
    assert old in s
    s = s.replace(old, new, 1)
open(p, "w").write(s)
