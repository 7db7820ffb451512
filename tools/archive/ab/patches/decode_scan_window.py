"""Candidate: decode scans a bitmap row of <= 16 aligned dwords with 16
independent scalar loads issued back to back (addresses clamped to the row's
last dword, so nothing outside the dwords the loop would read is touched),
folds the zero bytes into one 64-bit lost mask and walks it; longer rows keep
the dword loop."""
import sys
p = sys.argv[1]
s = open(p).read()
old = "    for (uint64_t a = rowaddr & ~3ull; a < end; a += 4) {"
new = """    const uint64_t a0 = rowaddr & ~3ull, alast = (end - 1) & ~3ull;
    if (alast - a0 < 64) {
      uint64_t lost = 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const uint64_t aq = a0 + 4ull * q < alast ? a0 + 4ull * q : alast;
        const uint32_t w = *(const_u32_as4)aq;
        const uint32_t z = ~(((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w) & 0x80808080u;
        const uint64_t nib = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
        lost |= nib << (4 * q);
      }
      lost >>= (uint32_t)(rowaddr - a0);
      if (g.k < 64) lost &= (1ull << g.k) - 1;
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
