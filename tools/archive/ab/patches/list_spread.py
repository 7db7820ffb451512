"""DIAGNOSTIC: work-list decode with the list walked alternately from its two
halves (item q -> q/2 or n/2 + q/2), so consecutive items come from stripes
half a batch apart: tests whether class tiles beat list tiles at half the
classes lost because their working tiles are spread over more stripes."""
import sys
p = sys.argv[1]
s = open(p).read()
old = """    const uint32_t item = *(const_u32_as4)(items + t / g.tiles_per_block);"""
assert old in s
s = s.replace(old, """    const uint64_t n = g.total_tiles / g.tiles_per_block, q = t / g.tiles_per_block;
    const uint64_t qq = (q & 1) ? (n + 1) / 2 + q / 2 : q / 2;
    const uint32_t item = *(const_u32_as4)(items + qq);""", 1)
open(p, "w").write(s)
