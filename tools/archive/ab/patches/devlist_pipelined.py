"""Candidate: software-pipelined grid-stride walk for decode_devlist_kernel.

On CDNA the vector-memory counter is in order and counts stores too, so in a
grid-stride loop written tile by tile -- loads(t), XOR, store(t), loads(t+G),
... -- the wait for loads(t+G) also waits for store(t) to be acknowledged
(the ISA shows `s_waitcnt vmcnt(7)` right after the next tile's first loads):
every iteration pays a store's round trip, which a one-workgroup-per-tile
launch never does (the wave ends after issuing its store).  Here the next
tile's loads are issued BEFORE the current tile's store, so the wait for them
leaves the youngest store outstanding.  Whole tiles only (bs a multiple of the
tile), compiled member counts; anything else takes the original loop.

    tools/ab/build_variant.sh devpipe tools/ab/patches/devlist_pipelined.py
"""
import os
import sys

p = sys.argv[1]
prefetch = os.environ.get("XEC_DEVPIPE_PREFETCH", "0") == "1"
s = open(p).read()

old = '''  if (*(const_i32_as4)g.gate != 0) return;
  const uint64_t total = (uint64_t)*(const_u32_as4)list * g.tiles_per_block;
  const uint32_t* entries = list + kDevListHeader;
  for (uint64_t t0 = blockIdx.x; t0 < total; t0 += gridDim.x) {'''
new = '''  if (*(const_i32_as4)g.gate != 0) return;
  const uint64_t total = (uint64_t)*(const_u32_as4)list * g.tiles_per_block;
  const uint32_t* entries = list + kDevListHeader;
  if constexpr (NM > 0 && U == 1 && NT) {
    if (g.bs % ((uint64_t)T * 16) == 0) {
      const uint32_t m = (uint32_t)g.m;
      const uint64_t stride = g.m * g.bs;
      uint64_t t0 = blockIdx.x;
      if (t0 >= total) return;
      // addresses of tile t: member pointer base, parity, destination
      auto where = [&](uint64_t t0_, const uint8_t*& base, const uint8_t*& sub, int& subst,
                       uint8_t*& dst, uint64_t& off) {
        const uint64_t t = total - 1 - t0_;
        const uint32_t item = *(const_u32_as4)(entries + t / g.tiles_per_block);
        const uint64_t chunk = t % g.tiles_per_block;
        const uint64_t c = item >> 8;
        const uint32_t i = item & 0xFFu;
        const uint32_t j = i % m, r = i / m;
        uint8_t* b = data + (c * g.k + j) * g.bs;
        base = b;
        sub = parity + (c * g.m + j) * g.bs;
        subst = (int)r;
        dst = b + (uint64_t)r * stride;
        off = (chunk * (uint64_t)T + threadIdx.x) * 16;
      };
      const uint8_t* base;
      const uint8_t* sub;
      int subst;
      uint8_t* dst;
      uint64_t off;
      where(t0, base, sub, subst, dst, off);
      u32x4 v[NM];
      {
        const uint8_t* q = base + off;
#pragma unroll
        for (int r = 0; r < NM; ++r, q += stride) v[r] = ld16<true>(r == subst ? sub + off : q);
      }
      for (;;) {
        u32x4 acc = v[0];
#pragma unroll
        for (int r = 1; r < NM; ++r) acc ^= v[r];
        uint8_t* cur_dst = dst;
        const uint64_t cur_off = off;
        const uint64_t n0 = t0 + gridDim.x;
        const bool more = n0 < total;
        if (more) {  // next tile's loads before this tile's store
          t0 = n0;
          where(t0, base, sub, subst, dst, off);
          const uint8_t* q = base + off;
#pragma unroll
          for (int r = 0; r < NM; ++r, q += stride) v[r] = ld16<true>(r == subst ? sub + off : q);
        }
        st16_block<true, kDecodeStoreAux>(cur_dst, cur_off, acc);
        if (!more) break;
      }
      return;
    }
  }
  for (uint64_t t0 = blockIdx.x; t0 < total; t0 += gridDim.x) {'''
if prefetch:  # the next tile's work item loaded one tile ahead of its data loads
    new = new.replace('''      auto where = [&](uint64_t t0_, const uint8_t*& base, const uint8_t*& sub, int& subst,
                       uint8_t*& dst, uint64_t& off) {
        const uint64_t t = total - 1 - t0_;
        const uint32_t item = *(const_u32_as4)(entries + t / g.tiles_per_block);''', '''      auto item_of = [&](uint64_t t0_) -> uint32_t {
        return t0_ < total ? *(const_u32_as4)(entries + (total - 1 - t0_) / g.tiles_per_block) : 0u;
      };
      uint32_t item_ahead = item_of(blockIdx.x + gridDim.x);
      auto where = [&](uint64_t t0_, const uint8_t*& base, const uint8_t*& sub, int& subst,
                       uint8_t*& dst, uint64_t& off, uint32_t item) {
        const uint64_t t = total - 1 - t0_;''')
    new = new.replace('''      where(t0, base, sub, subst, dst, off);
      u32x4 v[NM];''', '''      where(t0, base, sub, subst, dst, off, item_of(t0));
      u32x4 v[NM];''')
    new = new.replace('''        if (more) {  // next tile's loads before this tile's store
          t0 = n0;
          where(t0, base, sub, subst, dst, off);''', '''        if (more) {  // next tile's loads before this tile's store
          t0 = n0;
          const uint32_t it = item_ahead;
          item_ahead = item_of(t0 + gridDim.x);
          where(t0, base, sub, subst, dst, off, it);''')
    assert "item_ahead = item_of(t0 + gridDim.x)" in new
assert old in s
s = s.replace(old, new, 1)
open(p, "w").write(s)
