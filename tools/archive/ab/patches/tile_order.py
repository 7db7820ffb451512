"""Candidate tile orders (XEC_TILE_ORDER at patch time), replacing the product's
t = total-1-t0 in both kernels:
  fwd       t = t0
  halves    even workgroups walk from the front, odd ones from the back
  chunkrev  stripes (and classes) in order, the 1 KiB chunks of a block reversed
  striperev stripes reversed, chunks of a block in order
  skewhalf / skew37  the product order with each block's column walk rotated by
            half a block / 37 chunks per (stripe, class)"""
import os
import sys
p = sys.argv[1]
order = os.environ["XEC_TILE_ORDER"]
expr = {
    "fwd": "t0",
    "halves": "(t0 & 1) ? g.total_tiles - 1 - (t0 >> 1) : (t0 >> 1)",
    "chunkrev": "(t0 / g.tiles_per_block) * g.tiles_per_block + (g.tiles_per_block - 1 - t0 % g.tiles_per_block)",
    "striperev": "(g.total_tiles / g.tiles_per_block - 1 - t0 / g.tiles_per_block) * g.tiles_per_block + t0 % g.tiles_per_block",
    # the product's reverse order, with each block's column walk started at a
    # per-(stripe, class) offset so concurrent stripes touch different columns
    "skewhalf": "(g.total_tiles - 1 - t0) / g.tiles_per_block * g.tiles_per_block + ((g.total_tiles - 1 - t0) % g.tiles_per_block + ((g.total_tiles - 1 - t0) / g.tiles_per_block) * (g.tiles_per_block / 2)) % g.tiles_per_block",
    "skew37": "(g.total_tiles - 1 - t0) / g.tiles_per_block * g.tiles_per_block + ((g.total_tiles - 1 - t0) % g.tiles_per_block + ((g.total_tiles - 1 - t0) / g.tiles_per_block) * 37) % g.tiles_per_block",
}[order]
s = open(p).read()
old_e = "    const uint64_t t = g.total_tiles - 1 - t0;\n    const TileCoord tc = tile_coord(t, g);"
assert old_e in s
s = s.replace(old_e, f"    const uint64_t t = {expr};\n    const TileCoord tc = tile_coord(t, g);", 1)
old_d = "    const uint64_t t = g.total_tiles - 1 - t0;  // from the end of the batch, as encode"
assert old_d in s
s = s.replace(old_d, f"    const uint64_t t = {expr};", 1)
open(p, "w").write(s)
