"""Candidate: the encode/decode 16-byte stores with another cache policy
(gfx950 buffer aux bits: sc0 = 1, nt = 2, sc1 = 16).  The policy value is
taken from the XEC_STORE_AUX environment variable at patch time."""
import os
import sys
p = sys.argv[1]
aux = int(os.environ["XEC_STORE_AUX"], 0)
s = open(p).read()
old = "__builtin_amdgcn_raw_buffer_store_b128(v, rs, (uint32_t)off, 0, 2);"
assert old in s
s = s.replace(old, f"__builtin_amdgcn_raw_buffer_store_b128(v, rs, (uint32_t)off, 0, {aux});", 1)
open(p, "w").write(s)
