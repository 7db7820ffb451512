"""DIAGNOSTIC ONLY (wrong for any other erasure pattern): decode takes the lost
block of stripe c as (7c) mod k -- the bench pattern -- instead of scanning the
bitmap row, to price the scan."""
import sys
p = sys.argv[1]
s = open(p).read()
a = s.index("    for (uint64_t a = rowaddr & ~3ull; a < end; a += 4) {")
b = s.index("\n  }\n}\n", a)
s = s[:a] + """    (void)end;
    {
      const uint32_t i = (uint32_t)((7 * c) % g.k);
      const uint32_t j = i % m, r = i / m;
      uint8_t* base = sdata + (uint64_t)j * g.bs;
      xor_members<NM, U, NT, T>(base, stride, spar + (uint64_t)j * g.bs, (int)r,
                                base + (uint64_t)r * stride, off, g.bs, nm);
    }""" + s[b:]
open(p, "w").write(s)
