"""Candidate: each one-wave workgroup rebuilds CB consecutive 1 KiB chunks of
one class, one chunk after another with the product's loads in flight (all NM
members of a chunk), and stores the CB results together at the end: one 4 KiB
burst from one wave instead of four 1 KiB stores from four workgroups on four
XCDs.  Write-only streams run 1.4x faster with 4 KiB per workgroup than with
1 KiB (tools/lab/read_probe.hip, profiles/r03j; round 1's --wburst); earlier
4 KiB tiles changed the read side as well (256-thread tiles, members taken
G at a time over 4 KiB) and lost 1-4 %.  Here the read side keeps the
product's per-chunk shape.

Applies to encode_kernel and decode_arglist_kernel (configs 3 and 2: lists of
<= 1,024 lost blocks) for compiled member counts and U = 1; everything else
is the product.  Patch-time environment:
  XEC_CB=4    chunks per workgroup
  XEC_CB_SB=1 a scheduling barrier after each chunk's XOR (no chunk's loads
              hoisted above the previous chunk's reduction: exactly the
              product's loads in flight)

    XEC_CB=4 tools/ab/build_variant.sh cb4 tools/ab/patches/chunk_batch.py
"""
import os
import sys

p = sys.argv[1]
s = open(p).read()
CB = int(os.environ.get("XEC_CB", "4"))
SB = os.environ.get("XEC_CB_SB", "0") == "1"

helper = r'''
// ---- candidate: CB chunks per workgroup, stores batched (chunk_batch.py) ----
constexpr int kCB = %d;
template <int NM, bool NT, int T, int SAUX>
__device__ __forceinline__ void xor_chunks_batched(const uint8_t* base, uint64_t stride,
                                                   const uint8_t* sub, int subst, uint8_t* dst,
                                                   uint64_t sg, uint64_t tpb, uint64_t bs) {
  u32x4 res[kCB];
  uint64_t offs[kCB];
#pragma unroll
  for (int q = 0; q < kCB; ++q) {
    const uint64_t chunk = sg * kCB + (kCB - 1 - q);  // chunks walked downwards, as the product
    offs[q] = (chunk * (uint64_t)T + threadIdx.x) * 16;
    if (chunk >= tpb || offs[q] >= bs) { offs[q] = ~0ull; continue; }
    u32x4 v[NM];
    const uint8_t* pp = base + offs[q];
    const uint8_t* ps = sub + offs[q];
#pragma unroll
    for (int r = 0; r < NM; ++r, pp += stride) v[r] = ld16<NT>(r == subst ? ps : pp);
    if constexpr (NM >= 32) __builtin_amdgcn_sched_barrier(0);
    u32x4 acc = v[0];
#pragma unroll
    for (int r = 1; r < NM; ++r) acc ^= v[r];
    res[q] = acc;
    %s
  }
  asm volatile("" ::: "memory");
#pragma unroll
  for (int q = 0; q < kCB; ++q)
    if (offs[q] != ~0ull) st16_block<NT, SAUX>(dst, offs[q], res[q]);
}
''' % (CB, "__builtin_amdgcn_sched_barrier(0);" if SB else "")

anchor = "// ---------------------------------------------------------------------------\n// encode: parity[c][j]"
assert anchor in s
s = s.replace(anchor, helper + anchor, 1)

old_enc = '''  for (uint64_t t0 = blockIdx.x; t0 < g.total_tiles; t0 += gridDim.x) {
    // tiles are walked from the end of the batch (kReverse note above)
    const uint64_t t = g.total_tiles - 1 - t0;
    const TileCoord tc = tile_coord(t, g);'''
new_enc = '''  if constexpr (NM > 0 && U == 1) {
    const uint64_t tpb = g.tiles_per_block, sgpb = (tpb + kCB - 1) / kCB;
    const uint64_t total = g.S * g.m * sgpb;
    for (uint64_t t0 = blockIdx.x; t0 < total; t0 += gridDim.x) {
      const uint64_t t = total - 1 - t0;
      const uint64_t sg = t % sgpb, cj = t / sgpb, j = cj % g.m, c = cj / g.m;
      xor_chunks_batched<NM, NT, T, kEncodeStoreAux>(data + (c * g.k + j) * g.bs, g.m * g.bs,
                                                     nullptr, -1, parity + (c * g.m + j) * g.bs,
                                                     sg, tpb, g.bs);
    }
    return;
  }
  for (uint64_t t0 = blockIdx.x; t0 < g.total_tiles; t0 += gridDim.x) {
    // tiles are walked from the end of the batch (kReverse note above)
    const uint64_t t = g.total_tiles - 1 - t0;
    const TileCoord tc = tile_coord(t, g);'''
assert old_enc in s
s = s.replace(old_enc, new_enc, 1)

old_dec = '''                                                           Geometry g, ArgItems items) {
  for (uint64_t t0 = blockIdx.x; t0 < g.total_tiles; t0 += gridDim.x) {'''
new_dec = '''                                                           Geometry g, ArgItems items) {
  if constexpr (NM > 0 && U == 1) {
    const uint64_t tpb = g.tiles_per_block, sgpb = (tpb + kCB - 1) / kCB;
    const uint64_t total = g.total_tiles / tpb * sgpb;
    const uint64_t stride = g.m * g.bs;
    for (uint64_t t0 = blockIdx.x; t0 < total; t0 += gridDim.x) {
      const uint64_t t = total - 1 - t0;
      const uint32_t item = items.v[t / sgpb];
      const uint64_t c = item >> 8;
      const uint32_t i = item & 0xFFu, j = i % (uint32_t)g.m, r = i / (uint32_t)g.m;
      uint8_t* base = data + (c * g.k + j) * g.bs;
      xor_chunks_batched<NM, NT, T, kDecodeStoreAux>(base, stride, parity + (c * g.m + j) * g.bs,
                                                     (int)r, base + (uint64_t)r * stride,
                                                     t % sgpb, tpb, g.bs);
    }
    return;
  }
  for (uint64_t t0 = blockIdx.x; t0 < g.total_tiles; t0 += gridDim.x) {'''
assert old_dec in s
s = s.replace(old_dec, new_dec, 1)

old_ge = '''  const uint32_t grid = grid_for(g.total_tiles, ls.max_grid, ls.threads);
  const uint32_t lds = ls.lds_bytes;
  if (ls.threads == 256)
    return ls.nt ? enc_u'''
new_ge = '''  const uint64_t sg_tiles = g.total_tiles / g.tiles_per_block *
                            ((g.tiles_per_block + kCB - 1) / kCB);
  const bool batched = ls.unroll == 1 && g.nm > 0 && (g.nm & (g.nm - 1)) == 0 && g.nm <= 32;
  const uint32_t grid = grid_for(batched ? sg_tiles : g.total_tiles, ls.max_grid, ls.threads);
  const uint32_t lds = ls.lds_bytes;
  if (ls.threads == 256)
    return ls.nt ? enc_u'''
assert old_ge in s
s = s.replace(old_ge, new_ge, 1)

old_gd = '''  const ArgItems* a = tiling == kDecodeArgListTiles ? &args : nullptr;
  const uint32_t grid = grid_for(g.total_tiles, ls.max_grid, ls.threads);'''
new_gd = '''  const ArgItems* a = tiling == kDecodeArgListTiles ? &args : nullptr;
  const bool batched = tiling == kDecodeArgListTiles && ls.unroll == 1 && g.nm > 0 &&
                       (g.nm & (g.nm - 1)) == 0 && g.nm <= 32;
  const uint64_t sg_tiles = g.total_tiles / g.tiles_per_block *
                            ((g.tiles_per_block + kCB - 1) / kCB);
  const uint32_t grid = grid_for(batched ? sg_tiles : g.total_tiles, ls.max_grid, ls.threads);'''
assert old_gd in s
s = s.replace(old_gd, new_gd, 1)
open(p, "w").write(s)
