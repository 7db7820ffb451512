"""DIAGNOSTIC: work-list decode with an idle workgroup after every working one
(twice the grid; odd tiles exit at once), to test whether the idle tiles that
class tiles leave at half the classes lost are what makes them faster than
list tiles (DESIGN.md §3 Work-list tiles)."""
import sys
p = sys.argv[1]
s = open(p).read()
old = "  if (tiling == kDecodeListTiles) g.total_tiles = n_items * g.tiles_per_block;"
assert old in s
s = s.replace(old, "  if (tiling == kDecodeListTiles) g.total_tiles = 2 * n_items * g.tiles_per_block;", 1)
old = """    const uint64_t t = g.total_tiles - 1 - t0;  // from the end of the batch, as encode
    const uint64_t chunk = t % g.tiles_per_block;
    const uint32_t item = *(const_u32_as4)(items + t / g.tiles_per_block);"""
assert old in s
s = s.replace(old, """    const uint64_t t2 = g.total_tiles - 1 - t0;
    if (t2 & 1) continue;
    const uint64_t t = t2 >> 1;
    const uint64_t chunk = t % g.tiles_per_block;
    const uint32_t item = *(const_u32_as4)(items + t / g.tiles_per_block);""", 1)
open(p, "w").write(s)
