"""Candidate: encode stores parity `sc1` (not `nt`) when a class has 8
members; other member counts keep `nt`."""
import sys
p = sys.argv[1]
s = open(p).read()
old = """    xor_members<NM, U, NT, T, kEncodeStoreAux>(base, g.m * g.bs, nullptr, -1, dst, off, g.bs,
                                               (uint32_t)g.nm);"""
new = """    xor_members<NM, U, NT, T, NM == 8 ? kDecodeStoreAux : kEncodeStoreAux>(
        base, g.m * g.bs, nullptr, -1, dst, off, g.bs, (uint32_t)g.nm);"""
assert old in s
s = s.replace(old, new, 1)
open(p, "w").write(s)
