"""Candidate: for short classes (k/m <= 8) a decode tile rebuilds its stripe's
lost blocks G = 16/(k/m) at a time, all G*k/m loads in flight before the first
XOR, instead of one class reduction after another.  The bitmap row (k <= 60)
is folded into a 64-bit lost mask by the same dword scan."""
import sys
p = sys.argv[1]
s = open(p).read()

helper = r'''
// Rebuild up to G lost data blocks of one stripe over this lane's granule
// (idx[q] = block index, < 0 = unused slot): every G*NM load is issued before
// the first XOR.  m, bs, stride as in decode_kernel; off = the lane's offset.
template <int NM, int G, bool NT, int T>
__device__ __forceinline__ void rebuild_group(uint8_t* sdata, const uint8_t* spar,
                                              const int (&idx)[G], uint32_t m, uint64_t bs,
                                              uint64_t stride, uint64_t off) {
  u32x4 v[G][NM];
#pragma unroll
  for (int q = 0; q < G; ++q) {
    if (idx[q] < 0) continue;
    const uint32_t i = (uint32_t)idx[q], j = i % m, r = i / m;
    const uint8_t* p = sdata + (uint64_t)j * bs + off;
    const uint8_t* ps = spar + (uint64_t)j * bs + off;
#pragma unroll
    for (int rr = 0; rr < NM; ++rr, p += stride) v[q][rr] = ld16<NT>(rr == (int)r ? ps : p);
  }
#pragma unroll
  for (int q = 0; q < G; ++q) {
    if (idx[q] < 0) continue;
    const uint32_t i = (uint32_t)idx[q], j = i % m, r = i / m;
    u32x4 acc = v[q][0];
#pragma unroll
    for (int rr = 1; rr < NM; ++rr) acc ^= v[q][rr];
    st16_block<NT, kDecodeStoreAux>(sdata + (uint64_t)j * bs + (uint64_t)r * stride, off, acc);
  }
}

// ---------------------------------------------------------------------------
// decode: every lost data block'''
anchor = '''
// ---------------------------------------------------------------------------
// decode: every lost data block'''
assert anchor in s
s = s.replace(anchor, helper, 1)

old = '''    const uint64_t off = (chunk * (uint64_t)(T * U) + threadIdx.x) * 16;
    for (uint64_t a = rowaddr & ~3ull; a < end; a += 4) {'''
new = '''    const uint64_t off = (chunk * (uint64_t)(T * U) + threadIdx.x) * 16;
    if constexpr (NM > 0 && NM <= 8 && U == 1) {
      if (g.bs % (T * 16) == 0 && g.k <= 60) {
        const uint64_t a0 = rowaddr & ~3ull;
        uint64_t lost = 0;
        for (uint64_t a = a0; a < end; a += 4) {
          const uint32_t w = *(const_u32_as4)a;
          const uint32_t z = ~(((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w) & 0x80808080u;
          const uint64_t nib = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
          lost |= nib << (uint32_t)(a - a0);
        }
        lost = (lost >> (uint32_t)(rowaddr - a0)) & ((1ull << g.k) - 1);
        constexpr int G = 16 / NM;
        while (lost) {
          int idx[G];
#pragma unroll
          for (int q = 0; q < G; ++q) {
            idx[q] = lost ? (int)__builtin_ctzll(lost) : -1;
            lost &= lost - 1;
          }
          rebuild_group<NM, G, NT, T>(sdata, spar, idx, m, g.bs, stride, off);
        }
        continue;
      }
    }
    for (uint64_t a = rowaddr & ~3ull; a < end; a += 4) {'''
assert old in s
s = s.replace(old, new, 1)
open(p, "w").write(s)
