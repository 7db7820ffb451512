"""Candidate: one item per XCD.  Workgroups are dispatched round-robin over the
8 XCDs (workgroup b runs on XCD b % 8), so the 1 KiB chunks of one item (a
list entry, a stripe, a class) land on all eight XCDs and every CU works on
chunks of ~all the items in flight.  This permutes the tile index inside each
group of 8 consecutive items so that workgroups with the same b % 8 take the
chunks of one item: the chip-wide set of items in flight is unchanged, each
XCD (and CU) sees an eighth of it.  XEC_XPERM at patch time: "dec" (work-list
and stripe decode tiles), "all" (also encode and class tiles).

    XEC_XPERM=dec tools/ab/build_variant.sh xdec tools/ab/patches/xcd_items.py
"""
import os
import sys

p = sys.argv[1]
s = open(p).read()
mode = os.environ.get("XEC_XPERM", "dec")

helper = '''
// tile t of `total` (= items * tpb): within each group of 8 items, chunk-major
// so that t % 8 (= the XCD of its workgroup) selects the item (candidate).
__device__ __forceinline__ uint64_t xcd_perm(uint64_t t, uint64_t tpb, uint64_t total) {
  const uint64_t span = 8 * tpb;
  const uint64_t g0 = (t / span) * span;
  const uint64_t n = total - g0 < span ? (total - g0) / tpb : 8;
  const uint64_t w = t - g0;
  return g0 + (w % n) * tpb + w / n;
}

struct TileCoord {'''
s = s.replace("\nstruct TileCoord {", helper, 1)

rev = "const uint64_t t = g.total_tiles - 1 - t0;"
perm = "const uint64_t t = xcd_perm(g.total_tiles - 1 - t0, g.tiles_per_block, g.total_tiles);"
kernels = ["decode_kernel", "decode_list_kernel", "decode_arglist_kernel"]
if mode == "all":
    kernels += ["encode_kernel", "decode_class_kernel"]
for kname in kernels:
    i = s.index(f" void {kname}(")
    j = s.index(rev, i)
    s = s[:j] + perm + s[j + len(rev):]
open(p, "w").write(s)
