"""DIAGNOSTIC (wrong results by design; run ab.py with --no-check): where the
work-list decode tiles (rebuild_item: list, kernel-argument list and
device-list kernels) store the rebuilt chunk.  XEC_DIAG_DST at patch time:
  shadow  -- a separate allocation of the data buffer's size, same offset
  parity  -- the class's parity block, same column (the encode's write target)
  nostore -- no store (a never-true predicate keeps the loads alive)
Prices the in-place write at single-erasure m > 1 (2:1 .. 9:1 read/write).

    XEC_DIAG_DST=shadow tools/ab/build_variant.sh dshadow tools/ab/patches/decode_dst_diag.py
"""
import os
import sys

p = sys.argv[1]
s = open(p).read()
mode = os.environ.get("XEC_DIAG_DST", "shadow")
assert mode in ("shadow", "parity", "nostore")

old = '''  uint8_t* base = data + (c * g.k + j) * g.bs;
  const uint64_t off = (chunk * (uint64_t)(T * U) + threadIdx.x) * 16;
  xor_members<NM, U, NT, T, kDecodeStoreAux>(base, stride, parity + (c * g.m + j) * g.bs, (int)r,
                                             base + (uint64_t)r * stride, off, g.bs, nm);
}'''
assert old in s
if mode == "shadow":
    new = '''  uint8_t* base = data + (c * g.k + j) * g.bs;
  const uint64_t off = (chunk * (uint64_t)(T * U) + threadIdx.x) * 16;
  uint8_t* dst = g_diag_shadow + ((base + (uint64_t)r * stride) - data);
  xor_members<NM, U, NT, T, kDecodeStoreAux>(base, stride, parity + (c * g.m + j) * g.bs, (int)r,
                                             dst, off, g.bs, nm);
}'''
elif mode == "parity":
    new = '''  uint8_t* base = data + (c * g.k + j) * g.bs;
  const uint64_t off = (chunk * (uint64_t)(T * U) + threadIdx.x) * 16;
  uint8_t* dst = const_cast<uint8_t*>(parity) + (c * g.m + j) * g.bs;
  xor_members<NM, U, NT, T, kDecodeStoreAux>(base, stride, parity + (c * g.m + j) * g.bs, (int)r,
                                             dst, off, g.bs, nm);
}'''
else:
    new = '''  uint8_t* base = data + (c * g.k + j) * g.bs;
  const uint64_t off = (chunk * (uint64_t)(T * U) + threadIdx.x) * 16;
  const uint8_t* sub = parity + (c * g.m + j) * g.bs;
  if (NM > 0 && U == 1 && off < g.bs) {
    u32x4 acc = {0u, 0u, 0u, 0u};
    const uint8_t* q = base + off;
#pragma unroll
    for (int rr = 0; rr < (NM > 0 ? NM : 1); ++rr, q += stride)
      acc ^= ld16<NT>(rr == (int)r ? sub + off : q);
    if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u && acc.z == 0xF39CC060u && acc.w == 1u)
      st16_block<NT, kDecodeStoreAux>(base + (uint64_t)r * stride, off, acc);
    return;
  }
  xor_members<NM, U, NT, T, kDecodeStoreAux>(base, stride, sub, (int)r,
                                             base + (uint64_t)r * stride, off, g.bs, nm);
}'''
s = s.replace(old, new, 1)

if mode == "shadow":
    anchor = "namespace xec {\n"
    s = s.replace(anchor, anchor + "__device__ uint8_t* g_diag_shadow;\n", 1)
    old_l = '''  const uint32_t grid = grid_for(g.total_tiles, ls.max_grid, ls.threads);
  const uint32_t lds = ls.lds_bytes;
  if (ls.threads == 256)
    return ls.nt
               ? dec_u'''
    new_l = '''  {
    static uint8_t* shadow = nullptr;
    static uint64_t shadow_bytes = 0;
    const uint64_t need = g.S * g.k * g.bs;
    if (need > shadow_bytes) {
      if (shadow) (void)hipFree(shadow);
      if (hipMalloc(&shadow, need) != hipSuccess) return hipErrorOutOfMemory;
      shadow_bytes = need;
      hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_diag_shadow), &shadow, sizeof(shadow), 0,
                                       hipMemcpyHostToDevice);
      if (e != hipSuccess) return e;
    }
  }
  const uint32_t grid = grid_for(g.total_tiles, ls.max_grid, ls.threads);
  const uint32_t lds = ls.lds_bytes;
  if (ls.threads == 256)
    return ls.nt
               ? dec_u'''
    assert old_l in s
    s = s.replace(old_l, new_l, 1)
open(p, "w").write(s)
