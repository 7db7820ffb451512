"""Candidate: encode and class-tile decode walk the parity classes innermost.
The product's tile index runs chunk fastest, then class, then stripe, so the
tiles in flight together read the same class's k/m blocks (m*bs apart) -- at
m >= 2 and large blocks the one-failed-device geometry (DESIGN.md §3 *Which
block is lost*).  Here t -> (class j = t % m, chunk = (t / m) % tiles, stripe):
neighbouring tiles read the same column of every class of a stripe, i.e. all k
data blocks of the stripe at nearby columns, as the m = 1 encode (config 3,
0.87 of the spec) does.  m = 1 is unchanged."""
import sys
p = sys.argv[1]
s = open(p).read()
old = """  TileCoord tc;
  tc.chunk = t % g.tiles_per_block;
  const uint64_t cj = t / g.tiles_per_block;
  tc.j = cj % g.m;
  tc.c = cj / g.m;
  return tc;"""
new = """  TileCoord tc;
  tc.j = t % g.m;
  const uint64_t q = t / g.m;
  tc.chunk = q % g.tiles_per_block;
  tc.c = q / g.tiles_per_block;
  return tc;"""
assert old in s
s = s.replace(old, new, 1)
open(p, "w").write(s)
