// xec_scan.cpp -- host-side batch recoverability scan (xec_check_bitmap).
//
// Restates, for a whole batch in one pass, the reference's per-stripe
//   require_recovery  xorec_utils.hpp:144-149  (some DATA byte has bit 0 clear:
//                     popcount of byte & COMPLETE_DATA_BITMAP byte)
//   is_recoverable    xorec_utils.hpp:160-175  (per class, at most one ZERO byte
//                     among its data bytes and its parity byte)
// as evaluated over every stripe by xorec_gpu_decode (xorec_gpu_cmp.cu:75-81).
//
// Two forms:
//  * rows of <= 64 bytes (k + m <= 64) on an AVX2 host: one stripe per step,
//    zero-byte and bit-0-clear masks from two 32-byte loads (scan_rows_avx2),
//    ~2 ns per stripe (65536 stripes of cfg4 in ~140 us);
//  * otherwise: only bytes with bit 0 clear can matter to either rule, so the
//    scan finds those "candidates" (AVX2 or 8-byte SWAR) and visits each one;
//    candidates arrive in increasing position, so the stripe index advances
//    monotonically and the per-class marks are reset lazily per stripe.
// Compiled as plain host C++ (no HIP device pass), so target attributes and
// intrinsics are safe.  Per-call thread fan-out was tried and dropped: thread
// start-up cost more than the scan it split.
#include <cstdint>
#include <cstring>
#include <vector>

#include "xec.h"
#include "xec_internal.h"

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace {

struct Visitor {
  const uint8_t* bm;  // first byte of the first stripe this visitor scans
  size_t k, m, row;
  size_t cur_stripe = 0, row_start = 0;
  int need = 0;
  uint64_t lost_data = 0;  // zero data bytes seen
  uint64_t stripes_lost = 0;
  int64_t lost_class = -2;  // -2 none yet, -1 several, else the one class
  size_t last_lost_stripe = ~size_t(0);
  std::vector<uint32_t> mark;  // stripe+1 that last marked each class
  uint32_t* items = nullptr;   // optional work list (xec_scan_bitmap)
  uint64_t cap = 0;

  Visitor(const uint8_t* b, size_t k_, size_t m_) : bm(b), k(k_), m(m_), row(k_ + m_), mark(m_, 0) {}

  // false = a class lost two blocks (DecodeFailure)
  inline bool visit(size_t pos) {
    const uint8_t v = bm[pos];
    while (pos >= row_start + row) {
      row_start += row;
      ++cur_stripe;
    }
    const size_t i = pos - row_start;
    if (i < k) need = 1;
    if (v != 0) return true;  // bit 0 clear but nonzero: present for is_recoverable
    if (i < k) {
      if (lost_data < cap) items[lost_data] = xec_work_item(cur_stripe, i);
      ++lost_data;
      const int64_t c = static_cast<int64_t>(i % m);
      lost_class = lost_class == -2 ? c : lost_class == c ? c : -1;
      if (last_lost_stripe != cur_stripe) {
        last_lost_stripe = cur_stripe;
        ++stripes_lost;
      }
    }
    const size_t cls = i < k ? (m == 1 ? 0 : i % m) : i - k;
    const uint32_t tag = static_cast<uint32_t>(cur_stripe) + 1u;
    if (mark[cls] == tag) return false;
    mark[cls] = tag;
    return true;
  }
};

inline uint64_t load_u64(const uint8_t* p) {
  uint64_t w;
  std::memcpy(&w, p, 8);
  return w;
}

bool scan_swar(Visitor& v, size_t pos, size_t n) {
  constexpr uint64_t kOnes = 0x0101010101010101ull;
  for (; pos + 8 <= n; pos += 8) {
    uint64_t even = ~load_u64(v.bm + pos) & kOnes;  // bit 0 clear -> low bit of byte set
    while (even) {
      const int b = __builtin_ctzll(even) >> 3;
      if (!v.visit(pos + static_cast<size_t>(b))) return false;
      even &= even - 1;
    }
  }
  for (; pos < n; ++pos)
    if (!(v.bm[pos] & 1u) && !v.visit(pos)) return false;
  return true;
}

#if defined(__x86_64__)
__attribute__((target("avx2"))) bool scan_avx2(Visitor& v, size_t n) {
  const __m256i one = _mm256_set1_epi8(1);
  const __m256i zero = _mm256_setzero_si256();
  size_t pos = 0;
  for (; pos + 32 <= n; pos += 32) {
    const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(v.bm + pos));
    uint32_t mask = static_cast<uint32_t>(
        _mm256_movemask_epi8(_mm256_cmpeq_epi8(_mm256_and_si256(x, one), zero)));
    while (mask) {
      if (!v.visit(pos + static_cast<size_t>(__builtin_ctz(mask)))) return false;
      mask &= mask - 1;
    }
  }
  return scan_swar(v, pos, n);
}
#endif

bool scan_range(Visitor& v, size_t n) {
#if defined(__x86_64__)
  static const bool has_avx2 = __builtin_cpu_supports("avx2");
  if (has_avx2) return scan_avx2(v, n);
#endif
  return scan_swar(v, 0, n);
}

#if defined(__x86_64__)
// Per-stripe form for rows of at most 64 bytes (every practical k + m): two
// 32-byte loads give the row's zero-byte and bit-0-clear masks; the only
// branch is the (rare, predictable) ">= 2 zero bytes in one stripe" case,
// which checks classes with a bit set.  ~1.5 ns per stripe against ~5 ns for
// the per-candidate visitor, whose stripe bookkeeping mispredicts.
__attribute__((target("avx2,bmi,popcnt"))) int scan_rows_avx2(const uint8_t* bm, size_t S,
                                                             size_t k, size_t m, XecScan* out,
                                                             uint32_t* items, uint64_t cap,
                                                             bool speculative) {
  const size_t row = k + m;
  const uint64_t row_mask = row == 64 ? ~0ull : ((1ull << row) - 1);
  const uint64_t data_mask = (1ull << k) - 1;  // k < row <= 64
  uint8_t cls[64];
  for (size_t i = 0; i < row; ++i) cls[i] = static_cast<uint8_t>(i < k ? i % m : i - k);
  const __m256i one = _mm256_set1_epi8(1), zero = _mm256_setzero_si256();
  const size_t n = S * row;
  alignas(32) uint8_t pad[64];
  uint64_t need = 0, lost = 0, stripes_lost = 0, zd_or = 0;
  uint64_t listed_until = ~0ull;  // where a speculative list stopped (~0: it did not)
  for (size_t c = 0; c < S; ++c) {
    const uint8_t* r = bm + c * row;
    if (c * row + 64 > n) {  // last rows: never read past the caller's buffer
      std::memset(pad, 1, sizeof pad);
      std::memcpy(pad, r, row);
      r = pad;
    }
    const __m256i x0 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(r));
    const __m256i x1 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(r + 32));
    const uint64_t z =
        (static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(x0, zero))) |
         static_cast<uint64_t>(static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(x1, zero)))) << 32) &
        row_mask;
    const uint64_t e =
        (static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(_mm256_and_si256(x0, one), zero))) |
         static_cast<uint64_t>(static_cast<uint32_t>(
             _mm256_movemask_epi8(_mm256_cmpeq_epi8(_mm256_and_si256(x1, one), zero)))) << 32);
    need |= e & data_mask;
    uint64_t zd = z & data_mask;
    if (items != nullptr && lost < cap) {  // lost data blocks, in order, until the list is full
      for (uint64_t q = lost; zd; zd &= zd - 1, ++q)
        if (q < cap) items[q] = xec_work_item(c, static_cast<size_t>(__builtin_ctzll(zd)));
      zd = z & data_mask;
      // Speculative listing: every 32 rows, project the losses seen so far
      // over the batch, and stop writing a list the caller will not use (one
      // item costs ~1 ns, mostly the loop exit mispredicting on every row
      // with a loss: 1,024 of them were 1.3 us of an 8 MiB decode,
      // profiles/r06i).
      if (speculative && (c & 31) == 31) {
        const uint64_t seen = lost + static_cast<uint64_t>(__builtin_popcountll(zd));
        const uint64_t proj = seen * S / (c + 1);
        if (proj > cap + cap / 4 || (proj > S && 2 * proj >= S * m)) {
          listed_until = seen < cap ? seen : cap;
          items = nullptr;
        }
      }
    }
    lost += static_cast<uint64_t>(__builtin_popcountll(zd));
    stripes_lost += zd != 0;
    zd_or |= zd;  // every data position lost anywhere in the batch
    if (z & (z - 1)) {  // two or more zero bytes: they must be in different classes
      if (m == 1) return 0;
      uint64_t seen = 0, bits = z;
      while (bits) {
        const uint64_t bit = 1ull << cls[__builtin_ctzll(bits)];
        if (seen & bit) return 0;
        seen |= bit;
        bits &= bits - 1;
      }
    }
  }
  out->needs_recovery = need != 0;
  out->lost_data = lost;
  out->stripes_lost = stripes_lost;
  out->listed = listed_until != ~0ull ? listed_until : (lost < cap ? lost : cap);
  // one class iff every position in the union of the losses is in one class
  out->lost_class = -1;
  if (zd_or != 0) {
    const uint8_t c0 = cls[__builtin_ctzll(zd_or)];
    bool one = true;
    for (uint64_t b = zd_or; b && one; b &= b - 1) one = cls[__builtin_ctzll(b)] == c0;
    if (one) out->lost_class = c0;
  }
  return 1;
}
#endif

// ---- per-stripe verdicts (xec_decode_per_stripe) ---------------------------
// The reference CPU plugin decodes stripe by stripe (xorec_bm.cpp:43-58): an
// unrecoverable stripe fails alone and the others are rebuilt.  One verdict
// per stripe, and work items only for the stripes that are rebuilt.
struct StripeScan {
  uint8_t* codes;   // S verdicts (0 / 4), may be null
  uint32_t* items;  // may be null
  uint64_t cap;
  uint64_t n = 0, failures = 0;
  inline void emit(size_t c, uint64_t zd) {
    for (; zd; zd &= zd - 1, ++n)
      if (n < cap) items[n] = xec_work_item(c, static_cast<size_t>(__builtin_ctzll(zd)));
  }
};

void stripes_scalar(const uint8_t* bm, size_t S, size_t k, size_t m, StripeScan& o) {
  const size_t row = k + m;
  std::vector<uint8_t> hit(m);
  for (size_t c = 0; c < S; ++c) {
    const uint8_t* r = bm + c * row;
    bool need = false;
    for (size_t i = 0; i < k; ++i) need |= !(r[i] & 1u);  // require_recovery
    uint8_t code = 0;
    if (need) {  // is_recoverable: at most one zero byte per class
      for (size_t j = 0; j < m; ++j) hit[j] = r[k + j] == 0;
      for (size_t i = 0; i < k && code == 0; ++i)
        if (r[i] == 0) {
          if (hit[i % m]) code = 4;
          hit[i % m] = 1;
        }
      if (code == 0)
        for (size_t i = 0; i < k; ++i)
          if (r[i] == 0) {
            if (o.n < o.cap) o.items[o.n] = xec_work_item(c, i);
            ++o.n;
          }
    }
    o.failures += code != 0;
    if (o.codes) o.codes[c] = code;
  }
}

#if defined(__x86_64__)
__attribute__((target("avx2,bmi,popcnt"))) void stripes_avx2(const uint8_t* bm, size_t S,
                                                            size_t k, size_t m, StripeScan& o) {
  const size_t row = k + m;
  const uint64_t row_mask = row == 64 ? ~0ull : ((1ull << row) - 1);
  const uint64_t data_mask = (1ull << k) - 1;
  uint8_t cls[64];
  for (size_t i = 0; i < row; ++i) cls[i] = static_cast<uint8_t>(i < k ? i % m : i - k);
  const __m256i one = _mm256_set1_epi8(1), zero = _mm256_setzero_si256();
  const size_t n = S * row;
  alignas(32) uint8_t pad[64];
  for (size_t c = 0; c < S; ++c) {
    const uint8_t* r = bm + c * row;
    if (c * row + 64 > n) {
      std::memset(pad, 1, sizeof pad);
      std::memcpy(pad, r, row);
      r = pad;
    }
    const __m256i x0 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(r));
    const __m256i x1 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(r + 32));
    const uint64_t z =
        (static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(x0, zero))) |
         static_cast<uint64_t>(static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(x1, zero)))) << 32) &
        row_mask;
    const uint64_t e =
        (static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(_mm256_and_si256(x0, one), zero))) |
         static_cast<uint64_t>(static_cast<uint32_t>(
             _mm256_movemask_epi8(_mm256_cmpeq_epi8(_mm256_and_si256(x1, one), zero)))) << 32);
    uint8_t code = 0;
    if (e & data_mask) {
      if (z & (z - 1)) {
        uint64_t seen = 0, bits = z;
        for (; bits; bits &= bits - 1) {
          const uint64_t bit = 1ull << cls[__builtin_ctzll(bits)];
          if (seen & bit) {
            code = 4;
            break;
          }
          seen |= bit;
        }
      }
      if (code == 0) o.emit(c, z & data_mask);
    }
    o.failures += code != 0;
    if (o.codes) o.codes[c] = code;
  }
}
#endif

}  // namespace

xec_status xec_scan_stripes(const uint8_t* bm, size_t S, size_t k, size_t m, uint8_t* codes,
                            uint32_t* items, uint64_t cap, uint64_t* n_items,
                            uint64_t* failures) {
  if (k < 1 || m < 1 || k % m != 0) return XEC_INVALID_COUNTS;
  StripeScan o{codes, items, items ? cap : 0};
#if defined(__x86_64__)
  static const bool fast = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("bmi") &&
                           __builtin_cpu_supports("popcnt");
  if (fast && k + m <= 64 && S > 0)
    stripes_avx2(bm, S, k, m, o);
  else
#endif
    stripes_scalar(bm, S, k, m, o);
  if (n_items) *n_items = o.n;
  if (failures) *failures = o.failures;
  return XEC_SUCCESS;
}

// Also counts the zero (lost) data bytes and the stripes that have one and,
// when `items` is given, lists the first `cap` of them in batch order
// (xec_work_item).
xec_status xec_scan_bitmap(const uint8_t* bm, size_t S, size_t k, size_t m, XecScan* out,
                           uint32_t* items, uint64_t cap, bool speculative) {
  XecScan r;
  if (out) *out = r;
  if (k < 1 || m < 1 || k % m != 0) return XEC_INVALID_COUNTS;
#if defined(__x86_64__)
  static const bool fast = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("bmi") &&
                           __builtin_cpu_supports("popcnt");
  if (fast && k + m <= 64 && m <= 64 && S > 0) {
    if (!scan_rows_avx2(bm, S, k, m, &r, items, items ? cap : 0, speculative))
      return XEC_DECODE_FAILURE;
    if (out) *out = r;
    return XEC_SUCCESS;
  }
#endif
  Visitor v(bm, k, m);
  if (items != nullptr) {
    v.items = items;
    v.cap = cap;
  }
  if (!scan_range(v, S * (k + m))) return XEC_DECODE_FAILURE;
  r.needs_recovery = v.need;
  r.lost_data = v.lost_data;
  r.stripes_lost = v.stripes_lost;
  r.listed = v.lost_data < v.cap ? v.lost_data : v.cap;
  r.lost_class = v.lost_class >= 0 ? v.lost_class : -1;
  if (out) *out = r;
  return XEC_SUCCESS;
}

namespace {

void loss_masks_scalar(const uint8_t* bm, size_t S, size_t k, size_t m, uint32_t* masks) {
  const size_t row = k + m;
  for (size_t c = 0; c < S; ++c) {
    uint32_t mask = 0;
    for (size_t i = 0; i < k; ++i) mask |= static_cast<uint32_t>(bm[c * row + i] == 0) << i;
    masks[c] = mask;
  }
}

#if defined(__x86_64__)
// One 32-byte load per row covers its k <= 32 data bytes; the rows whose load
// would pass the end of the bitmap go through a padded copy.
__attribute__((target("avx2"))) void loss_masks_avx2(const uint8_t* bm, size_t S, size_t k,
                                                     size_t m, uint32_t* masks) {
  const size_t row = k + m, n = S * row;
  const uint32_t data_mask = k == 32 ? ~0u : ((1u << k) - 1);
  const __m256i zero = _mm256_setzero_si256();
  size_t c = 0;
  for (; c < S && c * row + 32 <= n; ++c) {
    const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(bm + c * row));
    masks[c] = static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(x, zero))) & data_mask;
  }
  if (c < S) loss_masks_scalar(bm + c * row, S - c, k, m, masks + c);
}
#endif

}  // namespace

void xec_loss_masks(const uint8_t* bm, size_t S, size_t k, size_t m, uint32_t* masks) {
#if defined(__x86_64__)
  static const bool fast = __builtin_cpu_supports("avx2");
  if (fast) {
    loss_masks_avx2(bm, S, k, m, masks);
    return;
  }
#endif
  loss_masks_scalar(bm, S, k, m, masks);
}

extern "C" xec_status xec_check_bitmap(const uint8_t* bm, size_t S, size_t k, size_t m,
                                       int* needs) {
  XecScan r;
  const xec_status st = xec_scan_bitmap(bm, S, k, m, &r, nullptr, 0);
  if (needs) *needs = r.needs_recovery;
  return st;
}

// The reference's erasure draw (select_lost_blocks, utils.cpp:100-127) with an
// explicit seed (include/xec.h): PCG32 (PCGRandom, utils.cpp:17-32) seeded
// RANDOM_SEED + seed on stream 1; each draw picks among the still-eligible
// block indices in increasing order and retires the drawn block's parity
// class.  The eligible list is compacted in place, so the draw sequence and
// the index it selects match the reference's erase_if over its vector.
extern "C" xec_status xec_select_lost_blocks(size_t k, size_t m, size_t lost, uint8_t* bm,
                                             uint64_t seed) {
  if (lost == 0) return XEC_SUCCESS;
  if (m == 0 || lost > m) return XEC_INVALID_COUNTS;
  if (bm == nullptr) return XEC_INVALID_SIZE;
  constexpr uint64_t kRandomSeed = 1896;  // RANDOM_SEED, utils.hpp:26
  uint64_t state = 0;
  const uint64_t inc = (1ull << 1) | 1ull;
  auto next = [&]() {
    const uint64_t old = state;
    state = old * 6364136223846793005ull + inc;
    const uint32_t xs = static_cast<uint32_t>(((old >> 18u) ^ old) >> 27u);
    const uint32_t rot = static_cast<uint32_t>(old >> 59u);
    return (xs >> rot) | (xs << ((0u - rot) & 31u));
  };
  (void)next();
  state += kRandomSeed + seed;
  (void)next();
  std::vector<uint32_t> eligible(k + m);
  for (size_t i = 0; i < eligible.size(); ++i) eligible[i] = static_cast<uint32_t>(i);
  size_t n = eligible.size();
  for (size_t d = 0; d < lost; ++d) {
    const uint32_t b = eligible[next() % n];
    bm[b] = 0;
    const size_t cls = b % m;
    size_t w = 0;
    for (size_t r = 0; r < n; ++r)
      if (eligible[r] % m != cls) eligible[w++] = eligible[r];
    n = w;
  }
  return XEC_SUCCESS;
}
