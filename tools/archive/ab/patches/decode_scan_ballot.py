"""Candidate: rows of <= 64 data bytes are read with one byte load per lane
and a wave ballot (one vector round trip) instead of the scalar dword loop."""
import sys
p = sys.argv[1]
s = open(p).read()
old = "    for (uint64_t a = rowaddr & ~3ull; a < end; a += 4) {"
new = """    if (g.k <= 64) {
      const uint32_t lane = threadIdx.x & 63u;
      const bool z = lane < g.k && reinterpret_cast<const uint8_t*>(rowaddr)[lane] == 0;
      uint64_t lost = __ballot(z);
      while (lost) {
        const uint32_t i = (uint32_t)__builtin_ctzll(lost);
        lost &= lost - 1;
        const uint32_t j = i % m, r = i / m;
        uint8_t* base = sdata + (uint64_t)j * g.bs;
        xor_members<NM, U, NT, T>(base, stride, spar + (uint64_t)j * g.bs, (int)r,
                                  base + (uint64_t)r * stride, off, g.bs, nm);
      }
      continue;
    }
    for (uint64_t a = rowaddr & ~3ull; a < end; a += 4) {"""
assert old in s
s = s.replace(old, new, 1)
open(p, "w").write(s)
