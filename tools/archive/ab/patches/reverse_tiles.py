"""Candidate: walk the tiles from the end of the batch to the start (workgroup
b takes tile total-1-b), for encode and decode alike."""
import sys
p = sys.argv[1]
s = open(p).read()
old_e = """  for (uint64_t t = blockIdx.x; t < g.total_tiles; t += gridDim.x) {
    const TileCoord tc = tile_coord(t, g);"""
new_e = """  for (uint64_t t0 = blockIdx.x; t0 < g.total_tiles; t0 += gridDim.x) {
    const uint64_t t = g.total_tiles - 1 - t0;
    const TileCoord tc = tile_coord(t, g);"""
assert old_e in s
s = s.replace(old_e, new_e, 1)
old_d = """  for (uint64_t t = blockIdx.x; t < g.total_tiles; t += gridDim.x) {
    const uint64_t chunk = t % g.tiles_per_block;"""
new_d = """  for (uint64_t t0 = blockIdx.x; t0 < g.total_tiles; t0 += gridDim.x) {
    const uint64_t t = g.total_tiles - 1 - t0;
    const uint64_t chunk = t % g.tiles_per_block;"""
assert old_d in s
s = s.replace(old_d, new_d, 1)
open(p, "w").write(s)
