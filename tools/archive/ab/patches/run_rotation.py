"""Candidate: the work-list decodes rotate a stripe's column walk by its place in
a run of consecutive stripes that lost a block of the SAME parity class, not by
its stripe index.  The automatic rotation (R = 3 per stripe, xec_api.cpp
decode_rotation) lifts one failed device +15 % at m >= 2 x 1 MiB, but a
rotation by stripe index costs the bench's pattern (class alternating from
stripe to stripe) up to 11 % and moves reference-style random losses only +2 %
(profiles/r04c, r04d).  By run position, neighbours of different classes keep
the same columns (the alternating geometry, the fastest one read_probe saw)
and neighbours of the same class get different ones; a run of 8 or more falls
back to the stripe index mod 8.  Driven with xec_set_rotation(R > 0) (the
host's automatic choice is unchanged here)."""
import sys
p = sys.argv[1]
s = open(p).read()


def rep(old, new):
    global s
    assert s.count(old) == 1, old
    s = s.replace(old, new)


rep("""template <int NM, int U, bool NT, int T>
__device__ __forceinline__ void rebuild_item(uint8_t* data, const uint8_t* __restrict__ parity,
                                             uint32_t item, uint64_t chunk, const Geometry& g) {""",
    """// the rotation index of list entry q: its place in the run of consecutive
// stripes before it whose entries lost a block of the same class (at most 7
// looked at; a longer run takes the stripe index mod 8)
template <typename Get>
__device__ __forceinline__ uint64_t run_index(uint64_t q, Get&& get, const Geometry& g) {
  if (g.rot == 0) return 0;
  const uint32_t item = get(q);
  const uint64_t c = item >> 8;
  const uint32_t m = (uint32_t)g.m, j = (item & 0xFFu) % m;
  uint64_t n = 0;
  while (n < 7 && q > n) {
    const uint32_t prev = get(q - n - 1);
    if ((uint64_t)(prev >> 8) + n + 1 != c || (prev & 0xFFu) % m != j) break;
    ++n;
  }
  return n == 7 ? c % 8 : n;
}

template <int NM, int U, bool NT, int T>
__device__ __forceinline__ void rebuild_item(uint8_t* data, const uint8_t* __restrict__ parity,
                                             uint32_t item, uint64_t chunk, const Geometry& g,
                                             uint64_t ridx) {""")
rep("""  const uint64_t off = (rotated(chunk, c, g) * (uint64_t)(T * U) + threadIdx.x) * 16;
  xor_members<NM, U, NT, T, kDecodeStoreAux>(base, stride, parity + (c * g.m + j) * g.bs, (int)r,""",
    """  const uint64_t off = (rotated(chunk, ridx, g) * (uint64_t)(T * U) + threadIdx.x) * 16;
  xor_members<NM, U, NT, T, kDecodeStoreAux>(base, stride, parity + (c * g.m + j) * g.bs, (int)r,""")
rep("""    const uint32_t item = *(const_u32_as4)(items + t / g.tiles_per_block);
    rebuild_item<NM, U, NT, T>(data, parity, item, t % g.tiles_per_block, g);""",
    """    const uint64_t q = t / g.tiles_per_block;
    const uint32_t item = *(const_u32_as4)(items + q);
    const uint64_t ridx =
        run_index(q, [&](uint64_t x) { return (uint32_t)*(const_u32_as4)(items + x); }, g);
    rebuild_item<NM, U, NT, T>(data, parity, item, t % g.tiles_per_block, g, ridx);""")
rep("""    rebuild_item<NM, U, NT, T>(data, parity, items.v[t / g.tiles_per_block],
                               t % g.tiles_per_block, g);""",
    """    const uint64_t q = t / g.tiles_per_block;
    const uint64_t ridx = run_index(q, [&](uint64_t x) { return items.v[x]; }, g);
    rebuild_item<NM, U, NT, T>(data, parity, items.v[q], t % g.tiles_per_block, g, ridx);""")
rep("""    const uint32_t item = *(const_u32_as4)(entries + t / g.tiles_per_block);
    rebuild_item<NM, U, NT, T>(data, parity, item, t % g.tiles_per_block, g);""",
    """    const uint32_t item = *(const_u32_as4)(entries + t / g.tiles_per_block);
    rebuild_item<NM, U, NT, T>(data, parity, item, t % g.tiles_per_block, g, item >> 8);""")
open(p, "w").write(s)
