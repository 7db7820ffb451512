"""CANDIDATE: kernel-argument work lists ordered by lost block index.

xec_decode's listing pass yields its items (c << 8 | i) in stripe order, so
with the bench's rotating erasures ((7c) mod k) the stripes in flight rebuild
blocks at different positions, while one failed device (the same i in every
stripe) decodes ~2.5 % faster at config 3 (profiles/r04c, r04d, r04zz).  This
orders the list by i (stable counting sort, k <= 256 buckets), stripes
ascending within each i, so the tiles in flight share a block position.
Applied to csrc/xec_api.cpp (XEC_PATCH_FILE=xec_api.cpp)."""
import sys
p = sys.argv[1]
s = open(p).read()
old = """      st = xec_scan_bitmap(h_bitmap, S, k, m, &scan, items, xec::kArgItems);
      if (st != XEC_SUCCESS) return st;
      g_tiling_used = XEC_TILING_ARG_LIST;"""
assert old in s
s = s.replace(old, """      st = xec_scan_bitmap(h_bitmap, S, k, m, &scan, items, xec::kArgItems);
      if (st != XEC_SUCCESS) return st;
      {
        uint32_t count[257] = {};
        uint32_t sorted[xec::kArgItems];
        const uint64_t n = scan.lost_data;
        for (uint64_t q = 0; q < n; ++q) ++count[(items[q] & 0xFFu) + 1];
        for (int b = 0; b < 256; ++b) count[b + 1] += count[b];
        for (uint64_t q = 0; q < n; ++q) sorted[count[items[q] & 0xFFu]++] = items[q];
        for (uint64_t q = 0; q < n; ++q) items[q] = sorted[q];
      }
      g_tiling_used = XEC_TILING_ARG_LIST;""", 1)
open(p, "w").write(s)
