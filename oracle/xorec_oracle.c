/*
 * xorec_oracle.c -- CPU restatement of the reference XOR-EC path.
 *
 * TEST INFRASTRUCTURE ONLY (see xorec_oracle.h): the checker for the HIP
 * path and the CPU baseline ("kind": "port") that bench.py times beside it.
 * Written from the reference's behaviour, not copied; each function cites
 * the reference file:line it restates.
 */
#include "xorec_oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* argument checks, src/xorec/xorec_utils.hpp:61-86                        */
/* Order matters and is kept: alignment first, then size, then counts.     */
/* ------------------------------------------------------------------------ */
int xo_check_args(const void* data, const void* parity, size_t bs, size_t k, size_t m) {
  if (((uintptr_t)data % XO_ALIGNMENT) != 0 || ((uintptr_t)parity % XO_ALIGNMENT) != 0)
    return XO_INVALID_ALIGNMENT;
  if (bs < XO_MIN_BLOCK_SIZE || bs % XO_BLOCK_SIZE_MULTIPLE != 0) return XO_INVALID_SIZE;
  if (k < 1 || m < 1 || k % m != 0) return XO_INVALID_COUNTS;
  return XO_SUCCESS;
}

/* require_recovery, xorec_utils.hpp:144-149: AND each data byte with the
 * all-ones COMPLETE_DATA_BITMAP (xorec.cpp:16-22) and popcount; recovery is
 * needed iff the count differs from k, i.e. iff some data byte has bit 0
 * clear. */
int xo_require_recovery(size_t k, const uint8_t* bitmap) {
  size_t count = 0;
  for (size_t i = 0; i < k; ++i) count += (size_t)(bitmap[i] & 1u);
  return count != k;
}

/* is_recoverable, xorec_utils.hpp:160-175: a parity class may lose at most
 * one block among {its data blocks} u {its parity block}. */
int xo_is_recoverable(size_t k, size_t m, const uint8_t* bitmap) {
  uint8_t stack_buf[256];
  uint8_t* needed = m <= sizeof stack_buf ? stack_buf : (uint8_t*)malloc(m);
  int ok = 1;
  for (size_t j = 0; j < m; ++j) needed[j] = bitmap[k + j] ? 0 : 1;
  for (size_t i = 0; i < k && ok; ++i) {
    if (bitmap[i]) continue;
    size_t cls = i % m;
    if (needed[cls]) ok = 0;
    needed[cls] = 1;
  }
  if (needed != stack_buf) free(needed);
  return ok;
}

/* dest ^= src over bytes (bs is a multiple of 256, so every reference
 * variant, xorec.hpp:174-273, covers the whole block and they agree).  Like
 * the reference's widest variant it moves 256 B per iteration as four 64-B
 * vectors (GCC vector extension; the clones let one binary pick AVX-512 /
 * AVX2 / SSE2 on whichever host runs it), so the CPU baseline times the same
 * instruction mix (tools/cpu_port_vs_ref.py). */
typedef uint64_t xo_v64 __attribute__((vector_size(64)));

__attribute__((target_clones("avx512f", "avx2", "default")))
static void xo_xor_into(uint8_t* __restrict dest, const uint8_t* __restrict src, size_t bytes) {
  xo_v64* __restrict d = (xo_v64*)__builtin_assume_aligned(dest, 64);
  const xo_v64* __restrict s = (const xo_v64*)__builtin_assume_aligned(src, 64);
  size_t n = bytes / 256;
  for (size_t w = 0; w < n; ++w, d += 4, s += 4) {
    const xo_v64 a0 = d[0] ^ s[0], a1 = d[1] ^ s[1], a2 = d[2] ^ s[2], a3 = d[3] ^ s[3];
    d[0] = a0;
    d[1] = a1;
    d[2] = a2;
    d[3] = a3;
  }
  /* bytes % 256 (never on the reference's checked sizes): word by word */
  uint64_t* dt = (uint64_t*)d;
  const uint64_t* st = (const uint64_t*)s;
  for (size_t w = 0; w < (bytes % 256) / 8; ++w) dt[w] ^= st[w];
}

/* xorec_encode, xorec.cpp:24-59: copy the first m data blocks into parity,
 * then fold data block i into parity block i % m for i = m..k-1. */
int xo_encode(const uint8_t* data, uint8_t* parity, size_t bs, size_t k, size_t m) {
  int err = xo_check_args(data, parity, bs, k, m);
  if (err != XO_SUCCESS) return err;
  memcpy(parity, data, m * bs);
  for (size_t i = m; i < k; ++i) xo_xor_into(parity + (i % m) * bs, data + i * bs, bs);
  return XO_SUCCESS;
}

/* xorec_decode, xorec.cpp:62-111.  No-op when no data block is lost; 4 when
 * a class lost two blocks; otherwise every lost data block i becomes
 * parity[i % m] ^ (XOR of the other data blocks of class i % m).  Lost parity
 * is never regenerated and parity is never written. */
int xo_decode(uint8_t* data, const uint8_t* parity, size_t bs, size_t k, size_t m,
              const uint8_t* bitmap) {
  int err = xo_check_args(data, parity, bs, k, m);
  if (err != XO_SUCCESS) return err;
  if (!xo_require_recovery(k, bitmap)) return XO_SUCCESS;
  if (!xo_is_recoverable(k, m, bitmap)) return XO_DECODE_FAILURE;
  for (size_t i = 0; i < k; ++i) {
    if (bitmap[i]) continue;
    uint8_t* rec = data + i * bs;
    memcpy(rec, parity + (i % m) * bs, bs);
    for (size_t j = i % m; j < k; j += m) {
      if (j == i) continue;
      xo_xor_into(rec, data + j * bs, bs);
    }
  }
  return XO_SUCCESS;
}

static void xo_set_threads(int threads) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#else
  (void)threads;
#endif
}

/* XorecBenchmark::encode, src/algorithms/xorec_bm.cpp:27-41 */
int xo_encode_batch(const uint8_t* data, uint8_t* parity, size_t S, size_t bs, size_t k,
                    size_t m, int threads) {
  int rc = 0;
  xo_set_threads(threads);
#pragma omp parallel for schedule(static)
  for (long c = 0; c < (long)S; ++c) {
    if (xo_encode(data + (size_t)c * k * bs, parity + (size_t)c * m * bs, bs, k, m) != XO_SUCCESS) {
#pragma omp atomic write
      rc = 1;
    }
  }
  return rc;
}

/* XorecBenchmark::decode, src/algorithms/xorec_bm.cpp:43-58 */
int xo_decode_batch(uint8_t* data, const uint8_t* parity, size_t S, size_t bs, size_t k,
                    size_t m, const uint8_t* bitmap, int threads) {
  int rc = 0;
  xo_set_threads(threads);
#pragma omp parallel for schedule(static)
  for (long c = 0; c < (long)S; ++c) {
    if (xo_decode(data + (size_t)c * k * bs, parity + (size_t)c * m * bs, bs, k, m,
                  bitmap + (size_t)c * (k + m)) != XO_SUCCESS) {
#pragma omp atomic write
      rc = 1;
    }
  }
  return rc;
}

/* xorec_gpu_decode's batch contract, src/xorec/xorec_gpu_cmp.cu:57-115 */
int xo_decode_batch_all_or_nothing(uint8_t* data, const uint8_t* parity, size_t S, size_t bs,
                                   size_t k, size_t m, const uint8_t* bitmap, int threads) {
  int err = xo_check_args(data, parity, bs, k, m);
  if (err != XO_SUCCESS) return err;
  int any = 0;
  for (size_t c = 0; c < S; ++c) {
    const uint8_t* b = bitmap + c * (k + m);
    if (xo_require_recovery(k, b)) any = 1;
    if (!xo_is_recoverable(k, m, b)) return XO_DECODE_FAILURE;
  }
  if (!any) return XO_SUCCESS;
  return xo_decode_batch(data, parity, S, bs, k, m, bitmap, threads) ? XO_DECODE_FAILURE
                                                                     : XO_SUCCESS;
}

/* ------------------------------------------------------------------------ */
/* synthetic data + hashing (SURVEY.md §8(c) known-answer convention)        */
/* ------------------------------------------------------------------------ */
static inline uint64_t xo_splitmix64_at(uint64_t seed, uint64_t n) {
  /* n-th output (0-based) of splitmix64 started from state `seed`. */
  uint64_t z = seed + (n + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void xo_fill_splitmix64(uint8_t* buf, size_t S, size_t stripe_bytes, uint64_t seed_base,
                        int threads) {
  size_t words = stripe_bytes / 8;
  xo_set_threads(threads);
#pragma omp parallel for schedule(static)
  for (long c = 0; c < (long)S; ++c) {
    uint64_t* w = (uint64_t*)(buf + (size_t)c * stripe_bytes);
    uint64_t seed = seed_base + (uint64_t)c;
    for (size_t n = 0; n < words; ++n) w[n] = xo_splitmix64_at(seed, n);
  }
}

uint64_t xo_fnv1a64(const uint8_t* p, size_t n, uint64_t h) {
  for (size_t i = 0; i < n; ++i) {
    h ^= p[i];
    h *= 0x100000001b3ull;
  }
  return h;
}

/* ------------------------------------------------------------------------ */
/* PCG32, src/utils/utils.cpp:17-32                                          */
/* ------------------------------------------------------------------------ */
uint32_t xo_pcg_next(xo_pcg* r) {
  uint64_t old = r->state;
  r->state = old * 6364136223846793005ull + r->inc;
  uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
  uint32_t rot = (uint32_t)(old >> 59u);
  return (xs >> rot) | (xs << ((-rot) & 31u));
}

void xo_pcg_init(xo_pcg* r, uint64_t seed, uint64_t seq) {
  r->state = 0;
  r->inc = (seq << 1u) | 1u;
  xo_pcg_next(r);
  r->state += seed;
  xo_pcg_next(r);
}

/* select_lost_blocks, src/utils/utils.cpp:100-127: draw `lost` indices from
 * the still-valid set; after each draw drop every index of the same parity
 * class so at most one block per class is lost. */
int xo_select_lost_blocks(size_t k, size_t m, size_t lost, uint8_t* bitmap, uint64_t seed) {
  if (lost == 0) return 0;
  if (lost > m) return -1;
  size_t tot = k + m;
  uint32_t* valid = (uint32_t*)malloc(tot * sizeof(uint32_t));
  size_t nvalid = tot;
  for (size_t i = 0; i < tot; ++i) valid[i] = (uint32_t)i;
  xo_pcg rng;
  xo_pcg_init(&rng, XO_RANDOM_SEED + seed, 1);
  for (size_t l = 0; l < lost; ++l) {
    size_t pick = xo_pcg_next(&rng) % nvalid;
    uint32_t idx = valid[pick];
    bitmap[idx] = 0;
    uint32_t cls = (uint32_t)(idx % m);
    size_t w = 0;
    for (size_t r = 0; r < nvalid; ++r)
      if (valid[r] % m != cls) valid[w++] = valid[r];
    nvalid = w;
  }
  free(valid);
  return 0;
}

/* write_validation_pattern, src/utils/utils.cpp:35-69 */
int xo_write_validation_pattern(uint8_t* block, size_t bytes, uint64_t seed) {
  if (bytes < 2) return -1;
  xo_pcg rng;
  xo_pcg_init(&rng, XO_RANDOM_SEED + seed, 1);
  if (bytes < 16) {
    uint8_t v = (uint8_t)xo_pcg_next(&rng);
    memset(block, v, bytes);
    return 0;
  }
  uint32_t crc = (uint32_t)bytes;
  uint32_t len = (uint32_t)bytes;
  memcpy(block + 4, &len, 4);
  for (size_t i = 8; i < bytes; ++i) {
    uint8_t v = (uint8_t)xo_pcg_next(&rng);
    block[i] = v;
    crc = (crc << 3) | (crc >> 29);
    crc += v;
  }
  memcpy(block, &crc, 4);
  return 0;
}

/* validate_block, src/utils/utils.cpp:72-97 */
int xo_validate_block(const uint8_t* block, size_t bytes) {
  if (bytes < 2) return 0;
  if (bytes < 16) {
    for (size_t i = 1; i < bytes; ++i)
      if (block[i] != block[0]) return 0;
    return 1;
  }
  uint32_t len, stored;
  memcpy(&len, block + 4, 4);
  if (len != (uint32_t)bytes) return 0;
  uint32_t crc = (uint32_t)bytes;
  for (size_t i = 8; i < bytes; ++i) {
    crc = (crc << 3) | (crc >> 29);
    crc += block[i];
  }
  memcpy(&stored, block, 4);
  return stored == crc;
}
