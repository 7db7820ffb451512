"""Candidate: each decode workgroup rebuilds TWO 1 KiB columns of the lost
block half a block apart (unroll 2 with the second granule at +bs/2), so a
column's in-place store is issued while the other column's loads -- far from
the stored address -- are in flight.  Blocks that are not a multiple of 2 KiB
keep the one-column tiles.  Encode is unchanged."""
import sys
p = sys.argv[1]
s = open(p).read()

def rep(old, new, n=1):
    global s
    assert s.count(old) >= n, old[:60]
    s = s.replace(old, new)

# runtime granule step for xor_members
rep("""                                            uint64_t off, uint64_t bs, uint32_t nm_rt) {
  constexpr uint64_t kStep = (uint64_t)T * 16;""",
    """                                            uint64_t off, uint64_t bs, uint32_t nm_rt,
                                            uint64_t kStep = (uint64_t)T * 16) {""")
# decode: far pair when U == 2
rep("""    const uint64_t off = (chunk * (uint64_t)(T * U) + threadIdx.x) * 16;
    for (uint64_t a = rowaddr & ~3ull; a < end; a += 4) {""",
    """    const bool far = U == 2 && g.bs % (2ull * T * 16) == 0;
    const uint64_t off = far ? (chunk * (uint64_t)T + threadIdx.x) * 16
                             : (chunk * (uint64_t)(T * U) + threadIdx.x) * 16;
    const uint64_t ustep = far ? g.bs / 2 : (uint64_t)T * 16;
    for (uint64_t a = rowaddr & ~3ull; a < end; a += 4) {""")
rep("""        xor_members<NM, U, NT, T>(base, stride, spar + (uint64_t)j * g.bs, (int)r,
                                  base + (uint64_t)r * stride, off, g.bs, nm);""",
    """        xor_members<NM, U, NT, T>(base, stride, spar + (uint64_t)j * g.bs, (int)r,
                                  base + (uint64_t)r * stride, off, g.bs, nm, ustep);""")
# launch: decode always unroll 2 far when the block allows it
rep("""  Geometry g = g_class;  // decode tiles are (stripe, chunk): see decode_kernel
  g.total_tiles = g.S * g.tiles_per_block;""",
    """  Geometry g = g_class;  // decode tiles are (stripe, chunk): see decode_kernel
  LaunchShape lsf = ls;
  if (ls.unroll == 1 && g.bs % (2ull * ls.threads * 16) == 0) {
    lsf.unroll = 2;
    g.tiles_per_block = g.bs / (2ull * ls.threads * 16);
  }
  g.total_tiles = g.S * g.tiles_per_block;""")
s = s.replace("""    return ls.nt ? dec_u<true, 256>(d_data, d_parity, d_bitmap, g, ls.unroll, grid, lds, s)
                 : dec_u<false, 256>(d_data, d_parity, d_bitmap, g, ls.unroll, grid, lds, s);
  return ls.nt ? dec_u<true, 64>(d_data, d_parity, d_bitmap, g, ls.unroll, grid, lds, s)
               : dec_u<false, 64>(d_data, d_parity, d_bitmap, g, ls.unroll, grid, lds, s);""",
"""    return ls.nt ? dec_u<true, 256>(d_data, d_parity, d_bitmap, g, lsf.unroll, grid, lds, s)
                 : dec_u<false, 256>(d_data, d_parity, d_bitmap, g, lsf.unroll, grid, lds, s);
  return ls.nt ? dec_u<true, 64>(d_data, d_parity, d_bitmap, g, lsf.unroll, grid, lds, s)
               : dec_u<false, 64>(d_data, d_parity, d_bitmap, g, lsf.unroll, grid, lds, s);""")
open(p, "w").write(s)
