"""DIAGNOSTIC (valid only for the bench pattern with one loss per stripe, every
stripe listed in order: entry e = stripe e, block (7e) mod k): the device-list
decode tile computes its work item instead of loading it (a dependent scalar
load per tile).  Prices the item load's latency on the list kernels.

    tools/ab/build_variant.sh noitem tools/ab/patches/list_noitem.py
"""
import sys

p = sys.argv[1]
s = open(p).read()
old = '''    const uint32_t item = *(const_u32_as4)(items + t / g.tiles_per_block);
    rebuild_item<NM, U, NT, T>(data, parity, item, t % g.tiles_per_block, g);'''
new = '''    const uint64_t e = t / g.tiles_per_block;
    const uint32_t item = (uint32_t)(e << 8) | (uint32_t)((7 * e) % g.k);
    rebuild_item<NM, U, NT, T>(data, parity, item, t % g.tiles_per_block, g);'''
assert old in s
s = s.replace(old, new, 1)
open(p, "w").write(s)
