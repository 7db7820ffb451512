"""EXPERIMENT (round 6): XCD-grouped tile order.  Workgroups are dispatched
round robin over the 8 XCDs (workgroup b on XCD b % 8), so neighbouring 1 KiB
chunks of a block -- adjacent tile indices -- land on different XCDs, and each
XCD writes 1 KiB pieces 8 KiB apart.  The write-only probe wrote 4 KiB
contiguous per one-wave workgroup at 6.61 TB/s against 4.77 for 1 KiB
(profiles/r03j).  This permutes the walk inside every group of 8*G workgroups
so that XCD x takes the G consecutive tiles x*G .. x*G+G-1 of the group, one
after another: each XCD streams G KiB contiguous.  G from XEC_XG (default 4);
a bijection on each whole group, identity on the ragged end, so every byte is
read and written exactly once.  Applied to encode and every decode tiling."""
import os
import re
import sys

path = sys.argv[1]
G = int(os.environ.get("XEC_XG", "4"))
s = open(path).read()
helper = f'''
__device__ __forceinline__ uint64_t xcd_group(uint64_t b, uint64_t total) {{
  constexpr uint64_t G = {G}, grp = 8 * G;
  if (b >= total - total % grp) return b;
  const uint64_t r = b % grp;
  return b - r + (r % 8) * G + r / 8;
}}
'''
anchor = "struct TileCoord {"
assert anchor in s
s = s.replace(anchor, helper + "\n" + anchor, 1)
n = 0
for old in ("const uint64_t t = g.total_tiles - 1 - t0;",):
    n += s.count(old)
    s = s.replace(old, "const uint64_t t = g.total_tiles - 1 - xcd_group(t0, g.total_tiles);")
assert n >= 5, n  # encode, stripe, class, list, arglist
open(path, "w").write(s)
print(f"xcd_group G={G}: {n} kernels")
