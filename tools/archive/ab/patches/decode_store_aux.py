"""Candidate: the decode kernels' rebuilt-block store with another cache
policy (gfx950 buffer aux bits: sc0 = 1, nt = 2, sc1 = 16; the product uses
sc1).  The value is taken from XEC_DEC_AUX at patch time."""
import os
import sys
p = sys.argv[1]
aux = int(os.environ["XEC_DEC_AUX"], 0)
s = open(p).read()
old = "constexpr int kDecodeStoreAux = 16;  // sc1"
assert old in s
s = s.replace(old, f"constexpr int kDecodeStoreAux = {aux};", 1)
open(p, "w").write(s)
