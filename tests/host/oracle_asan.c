/* oracle_asan.c -- the oracle's C restatement (oracle/xorec_oracle.c) under
 * AddressSanitizer + UBSan, as SURVEY.md §5 asks: exact-size 64-B aligned
 * buffers, the SURVEY.md §8(c) known-answer parity hashes, and
 * encode -> erase -> all-or-nothing decode round trips on random shapes.
 * Built and run by tests/test_host_sanitizers.py. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "xorec_oracle.h"

static uint8_t* alloc64(size_t n) {
  void* p = NULL;
  if (posix_memalign(&p, 64, n ? n : 1) != 0) abort();
  return (uint8_t*)p;
}

int main(void) {
  static const struct { size_t k, m, bs; uint64_t fnv; } ka[] = {
      {4, 1, 4096, 0xb2c6b787b51d553bull},  {8, 1, 65536, 0x7ed09decdded0a43ull},
      {32, 1, 4096, 0xf4816739ea1136a6ull}, {8, 4, 1024, 0xff5c7b96c04c0292ull}};
  for (size_t t = 0; t < sizeof ka / sizeof *ka; ++t) {
    uint8_t* d = alloc64(ka[t].k * ka[t].bs);
    uint8_t* p = alloc64(ka[t].m * ka[t].bs);
    xo_fill_splitmix64(d, 1, ka[t].k * ka[t].bs, XO_RANDOM_SEED, 1);
    if (xo_encode(d, p, ka[t].bs, ka[t].k, ka[t].m) != XO_SUCCESS) return 1;
    if (xo_fnv1a64(p, ka[t].m * ka[t].bs, 0xcbf29ce484222325ull) != ka[t].fnv) {
      printf("known answer %zu mismatch\n", t);
      return 1;
    }
    free(d);
    free(p);
  }
  xo_pcg rng;
  xo_pcg_init(&rng, 7, 1);
  for (int trial = 0; trial < 300; ++trial) {
    const size_t m = 1 + xo_pcg_next(&rng) % 8, k = m * (1 + xo_pcg_next(&rng) % 10);
    const size_t bs = 256 * (1 + xo_pcg_next(&rng) % 8), S = 1 + xo_pcg_next(&rng) % 6;
    uint8_t* d = alloc64(S * k * bs);
    uint8_t* p = alloc64(S * m * bs);
    uint8_t* ref = alloc64(S * k * bs);
    uint8_t* bm = alloc64(S * (k + m));
    xo_fill_splitmix64(d, S, k * bs, 100 + (uint64_t)trial, 2);
    memcpy(ref, d, S * k * bs);
    if (xo_encode_batch(d, p, S, bs, k, m, 2) != 0) return 1;
    memset(bm, 1, S * (k + m));
    const int bad_stripe = trial % 7 == 0 ? (int)(xo_pcg_next(&rng) % S) : -1;
    for (size_t c = 0; c < S; ++c) {
      if (xo_select_lost_blocks(k, m, xo_pcg_next(&rng) % (m + 1), bm + c * (k + m), c) < 0)
        return 1;
      if ((int)c == bad_stripe) bm[c * (k + m)] = bm[c * (k + m) + k] = 0;
      for (size_t i = 0; i < k; ++i)
        if (!bm[c * (k + m) + i]) memset(d + (c * k + i) * bs, 0, bs);
    }
    const int st = xo_decode_batch_all_or_nothing(d, p, S, bs, k, m, bm, 2);
    if (bad_stripe >= 0) {
      if (st != XO_DECODE_FAILURE) return 1;
    } else if (st != XO_SUCCESS || memcmp(d, ref, S * k * bs) != 0) {
      printf("round trip %d failed (st %d)\n", trial, st);
      return 1;
    }
    free(d);
    free(p);
    free(ref);
    free(bm);
  }
  printf("oracle_asan ok\n");
  return 0;
}
