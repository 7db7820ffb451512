// xec_validate.hip -- device-side validation payload and check.
//
// The reference's only correctness check is a per-block payload: random PCG
// bytes from offset 8, the block length (u32) at 4 and a rotate-add checksum
// (u32, crc = rotl(crc,3) + byte, seeded with the length) at 0
// (src/utils/utils.cpp:35-97), generated and validated on the host with a
// full device<->host copy each iteration (xorec_gpu_cmp_bm.cpp:25-37,91-104).
// Here both run where the data lives (generation: PCG32, utils.cpp:17-32, with
// state RANDOM_SEED + seed + block, stream 1; the wall-clock seed of the
// reference is replaced by an explicit one).
//
// Two kernel shapes, same results:
//  * lane per block (serial_*): one lane walks a whole block.  Used for the
//    pattern when there are enough blocks to fill the chip (>= kLaneBlocks),
//    and whenever the block does not tile into 128-byte segments.
//  * G lanes per block (wave_*<G>, 64/G blocks per wave): the lanes split the
//    checksum chain.  Past a serial head (bytes 8..127), a block is walked in
//    windows of G*128 bytes, lane j owning the 128 contiguous bytes at
//    window + 128 j.  rotl3 is multiplication by 8 modulo 2^32-1 and
//    8^128 == 1 there, so a lane's segment maps a start state x to x + S
//    (ones'-complement) where S is the segment's Horner sum -- unless an
//    addition carried out of 32 bits, which the ones'-complement form cannot
//    see (probability ~2^-25 per byte).  Each lane takes the speculated start
//    W + S_0 + ... + S_{j-1} (a scan over the group), runs the true chain from
//    it and checks that it ends where lane j+1 starts.  Lane 0 starts from the
//    exact state, so if every check passes every lane was exact; otherwise
//    the window is redone lane after lane.  Exact by construction; modelled
//    in Python in tests/crc_model.py, tests/test_crc_split.py.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "xec_kernels.h"

namespace xec {

namespace {

constexpr uint64_t kPcgMul = 6364136223846793005ull;
constexpr uint64_t kRandomSeed = 1896;  // RANDOM_SEED, utils.hpp:26

struct Pcg {
  uint64_t state, inc;
  __device__ uint32_t next() {
    const uint64_t old = state;
    state = old * kPcgMul + inc;
    const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    const uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((0u - rot) & 31u));
  }
  __device__ Pcg(uint64_t seed, uint64_t seq) : state(0), inc((seq << 1u) | 1u) {
    next();
    state += seed;
    next();
  }
};

__device__ __forceinline__ uint32_t rotl3(uint32_t x) { return (x << 3) | (x >> 29); }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// x + byte Q of w in one v_add_u32 with an SDWA byte select.  Written as asm
// so the byte extracts cannot be hoisted out of the chain (the scheduler would
// otherwise keep all 128 extracted bytes live, 120+ VGPRs).
#define XEC_ADD_BYTE(Q)                                                                   \
  __device__ __forceinline__ uint32_t add_byte##Q(uint32_t x, uint32_t w) {              \
    uint32_t r;                                                                          \
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "  \
        "src1_sel:BYTE_" #Q                                                              \
        : "=v"(r)                                                                        \
        : "v"(x), "v"(w));                                                               \
    return r;                                                                            \
  }
XEC_ADD_BYTE(0)
XEC_ADD_BYTE(1)
XEC_ADD_BYTE(2)
XEC_ADD_BYTE(3)
#undef XEC_ADD_BYTE

// The reference chain (utils.cpp:53-55) over one little-endian word.
__device__ __forceinline__ uint32_t word_chain(uint32_t x, uint32_t w) {
  x = add_byte0(rotl3(x), w);
  x = add_byte1(rotl3(x), w);
  x = add_byte2(rotl3(x), w);
  return add_byte3(rotl3(x), w);
}

__global__ __launch_bounds__(256) void serial_pattern_kernel(uint8_t* data, uint64_t nblocks,
                                                             uint64_t bs, uint64_t seed) {
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nblocks) return;
  uint8_t* blk = data + b * bs;
  Pcg rng(kRandomSeed + seed + b, 1);
  if (bs < 16) {
    const uint8_t v = (uint8_t)rng.next();
    for (uint64_t i = 0; i < bs; ++i) blk[i] = v;
    return;
  }
  uint32_t crc = (uint32_t)bs;
  uint64_t i = 8;
  if (bs % 16 == 0) {
    // bytes 8..15 first, then whole 16-byte granules
    uint32_t w[2] = {0, 0};
    for (int q = 0; q < 8; ++q) {
      const uint32_t v = rng.next() & 0xffu;
      w[q >> 2] |= v << (8 * (q & 3));
      crc = rotl3(crc) + v;
    }
    reinterpret_cast<uint32_t*>(blk)[2] = w[0];
    reinterpret_cast<uint32_t*>(blk)[3] = w[1];
    for (i = 16; i < bs; i += 16) {
      u32x4 g = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const uint32_t v = rng.next() & 0xffu;
        g[q >> 2] |= v << (8 * (q & 3));
        crc = rotl3(crc) + v;
      }
      *reinterpret_cast<u32x4*>(blk + i) = g;
    }
  } else {
    for (; i < bs; ++i) {
      const uint8_t v = (uint8_t)rng.next();
      blk[i] = v;
      crc = rotl3(crc) + v;
    }
  }
  const uint32_t len = (uint32_t)bs;
  for (int q = 0; q < 4; ++q) {
    blk[4 + q] = (uint8_t)(len >> (8 * q));
    blk[q] = (uint8_t)(crc >> (8 * q));
  }
}

__global__ __launch_bounds__(256) void serial_validate_kernel(const uint8_t* data,
                                                              uint64_t nblocks, uint64_t bs,
                                                              uint32_t* bad) {
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nblocks) return;
  const uint8_t* blk = data + b * bs;
  bool ok;
  if (bs < 2) {
    ok = false;
  } else if (bs < 16) {
    ok = true;
    for (uint64_t i = 1; i < bs; ++i) ok &= blk[i] == blk[0];
  } else {
    uint32_t len = 0, stored = 0;
    for (int q = 0; q < 4; ++q) {
      len |= (uint32_t)blk[4 + q] << (8 * q);
      stored |= (uint32_t)blk[q] << (8 * q);
    }
    uint32_t crc = (uint32_t)bs;
    uint64_t i = 8;
    if (bs % 16 == 0) {
      for (; i < 16; ++i) crc = rotl3(crc) + blk[i];
      for (; i < bs; i += 16) {
        const u32x4 g = *reinterpret_cast<const u32x4*>(blk + i);
#pragma unroll
        for (int c = 0; c < 4; ++c) crc = word_chain(crc, g[c]);
      }
    } else {
      for (; i < bs; ++i) crc = rotl3(crc) + blk[i];
    }
    ok = len == (uint32_t)bs && stored == crc;
  }
  if (!ok) atomicAdd(bad, 1u);
}

// ---- G lanes per block (a wave holds 64/G blocks) -----------------------------

constexpr int kSeg = 128;                     // bytes per lane per window
constexpr uint64_t kLaneBlocks = 1ull << 18;  // pattern: lane per block fills the chip from here

__device__ __forceinline__ uint32_t oc_add(uint32_t a, uint32_t b) {  // mod 2^32-1
  const uint32_t s = a + b;
  return s + (uint32_t)(s < a);
}
__device__ __forceinline__ uint32_t rotl12(uint32_t x) { return (x << 12) | (x >> 20); }

struct Segment {
  u32x4 g[kSeg / 16];
};

// Horner sum of the segment's bytes, sum 8^(kSeg-1-n) v_n mod 2^32-1, four
// bytes (one factor 8^4 = rotl12) per step.
__device__ __forceinline__ uint32_t seg_horner(const Segment& sg) {
  uint32_t s = 0;
#pragma unroll
  for (int t = 0; t < kSeg / 16; ++t)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t w = sg.g[t][c];
      // 8^3 b0 + 8^2 b1 + 8 b2 + b3 = 8 * dot4(bytes, (64, 8, 1, 0)) + b3
      const uint32_t v = (__builtin_amdgcn_udot4(w, 0x00010840u, 0u, false) << 3) + (w >> 24);
      s = oc_add(rotl12(s), v);
    }
  return s;
}

// ... and the reference chain over the segment from state x.
__device__ __forceinline__ uint32_t seg_chain(uint32_t x, const Segment& sg) {
#pragma unroll
  for (int t = 0; t < kSeg / 16; ++t)
#pragma unroll
    for (int c = 0; c < 4; ++c) x = word_chain(x, sg.g[t][c]);
  return x;
}

// Advance the checksum state W over one window of G segments; every lane of
// the group returns the state after the window.  `sub` = lane within the
// group; `active` = the lane's segment lies inside the block (inactive lanes
// are the group's tail and act as the identity).
template <int G>
__device__ uint32_t window_crc(uint32_t W, const Segment& sg, bool active, int sub) {
  const uint32_t S = active ? seg_horner(sg) : 0u;
  uint32_t incl = S;
#pragma unroll
  for (int d = 1; d < G; d <<= 1) {
    const uint32_t t = __shfl_up(incl, d, G);
    if (sub >= d) incl = oc_add(incl, t);
  }
  const uint32_t excl = __shfl_up(incl, 1, G);
  const uint32_t start = sub == 0 ? W : oc_add(W, excl);
  const uint32_t end = active ? seg_chain(start, sg) : start;
  const uint32_t next_start = __shfl_down(start, 1, G);
  if (__ballot(sub < G - 1 && end != next_start) == 0) return __shfl(end, G - 1, G);
  // a carry somewhere in the wave: every group walks its window lane after
  // lane from its exact state
  uint32_t cur = W;
  for (int j = 0; j < G; ++j) {
    const uint32_t e = active ? seg_chain(cur, sg) : cur;
    cur = __shfl(e, j, G);
  }
  return cur;
}

// Validation walks the whole block as segments 0.. of kSeg bytes.  Segment 0
// holds the 8-byte header (checksum, size) and then the first payload bytes;
// the chain starts at byte 8 from the size (utils.cpp:72-97).  Lane 0 takes
// segment 0 with its header words read as zero: eight zero bytes only rotate
// the state (rotl3 eight times is rotl 24, and adding 0 never carries), so a
// chain started at rotl(bs, 8) reaches exactly bs at byte 8 and continues as
// the reference's.  The header then costs one lane's segment, not a serial
// chain of 120 bytes that every lane of the wave walks first (round 3: that
// chain was as many instructions per wave as the whole split window at 4 KiB
// blocks).
__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return (x << 8) | (x >> 24); }

// Requires bs % kSeg == 0, bs >= 2 kSeg, 16-B aligned blocks; G >= the
// segments per block, or 64.  Windows of G*kSeg bytes.
template <int G>
__global__ __launch_bounds__(64) void wave_validate_kernel(const uint8_t* data, uint64_t nblocks,
                                                           uint64_t bs, uint32_t* bad) {
  constexpr int kBpw = 64 / G;  // blocks per wave
  constexpr uint64_t kWin = (uint64_t)G * kSeg;
  const int sub = threadIdx.x % G;
  for (uint64_t b0 = (uint64_t)blockIdx.x * kBpw; b0 < nblocks; b0 += (uint64_t)gridDim.x * kBpw) {
    const uint64_t b = b0 + threadIdx.x / G;
    const bool valid = b < nblocks;
    const uint8_t* blk = data + (valid ? b : b0) * bs;
    auto load = [&](Segment& sg, uint64_t base) {
      const uint64_t off = base + (uint64_t)sub * kSeg;
      const u32x4* src = reinterpret_cast<const u32x4*>(blk + (valid && off < bs ? off : 0));
#pragma unroll
      for (int t = 0; t < kSeg / 16; ++t) sg.g[t] = src[t];
    };
    Segment cur;
    load(cur, 0);
    if (sub == 0) {  // the header reads as zero (above)
      cur.g[0][0] = 0u;
      cur.g[0][1] = 0u;
    }
    uint32_t W = rotl8((uint32_t)bs);
    if constexpr (G < 64) {  // G covers the block: one window
      W = window_crc<G>(W, cur, valid && (uint64_t)sub * kSeg < bs, sub);
    } else {  // the next window's segment is in flight while this one is reduced
      Segment nxt;
      for (uint64_t base = 0; base < bs; base += kWin) {
        if (base + kWin < bs) load(nxt, base + kWin);
        W = window_crc<G>(W, cur, base + (uint64_t)sub * kSeg < bs, sub);
        cur = nxt;
      }
    }
    if (valid && sub == 0) {
      const uint32_t* hdr = reinterpret_cast<const uint32_t*>(blk);
      if (!(hdr[1] == (uint32_t)bs && hdr[0] == W)) atomicAdd(bad, 1u);
    }
  }
}

// PCG32 advance by `delta` steps (log-time LCG jump).
__device__ uint64_t pcg_advance(uint64_t state, uint64_t delta, uint64_t inc) {
  uint64_t acc_mult = 1, acc_plus = 0, cur_mult = kPcgMul, cur_plus = inc;
  while (delta) {
    if (delta & 1) {
      acc_mult *= cur_mult;
      acc_plus = acc_plus * cur_mult + cur_plus;
    }
    cur_plus = (cur_mult + 1) * cur_plus;
    cur_mult *= cur_mult;
    delta >>= 1;
  }
  return acc_mult * state + acc_plus;
}

// Same layout as wave_validate_kernel; each lane generates its segment of a
// window from the PCG state jumped to the segment's first byte (byte i of a
// block is output number i-8).
template <int G>
__global__ __launch_bounds__(64) void wave_pattern_kernel(uint8_t* data, uint64_t nblocks,
                                                          uint64_t bs, uint64_t seed) {
  constexpr int kBpw = 64 / G;
  constexpr uint64_t kWin = (uint64_t)G * kSeg;
  const int sub = threadIdx.x % G;
  for (uint64_t b0 = (uint64_t)blockIdx.x * kBpw; b0 < nblocks; b0 += (uint64_t)gridDim.x * kBpw) {
    const uint64_t b = b0 + threadIdx.x / G;
    const bool valid = b < nblocks;
    uint8_t* blk = data + (valid ? b : b0) * bs;
    Pcg rng(kRandomSeed + seed + b, 1);
    const uint64_t state0 = rng.state;
    uint32_t W = (uint32_t)bs;
    for (int i = 2; i < kSeg / 4; ++i) {  // head, bytes 8..kSeg-1
      uint32_t x = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) x |= (rng.next() & 0xffu) << (8 * q);
      W = word_chain(W, x);
      if (valid && sub == 0) reinterpret_cast<uint32_t*>(blk)[i] = x;
    }
    rng.state = pcg_advance(state0, (uint64_t)kSeg - 8 + (uint64_t)sub * kSeg, rng.inc);
    for (uint64_t base = kSeg; base < bs; base += kWin) {
      const uint64_t off = base + (uint64_t)sub * kSeg;
      const bool active = valid && off < bs;
      Segment sg;
#pragma unroll
      for (int t = 0; t < kSeg / 16; ++t) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          uint32_t x = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) x |= (rng.next() & 0xffu) << (8 * q);
          asm volatile("" : "+v"(x));  // in order: keeps the scheduler from holding 128 PCG states
          sg.g[t][c] = x;
        }
      }
      if (active) {
        u32x4* dst = reinterpret_cast<u32x4*>(blk + off);
#pragma unroll
        for (int t = 0; t < kSeg / 16; ++t) dst[t] = sg.g[t];
      }
      W = window_crc<G>(W, sg, active, sub);
      if (base + kWin < bs) rng.state = pcg_advance(rng.state, kWin - kSeg, rng.inc);
    }
    if (valid && sub == 0) {
      reinterpret_cast<uint32_t*>(blk)[0] = W;
      reinterpret_cast<uint32_t*>(blk)[1] = (uint32_t)bs;
    }
  }
}

// Lanes per block, rounded up to a power of two, at most a wave: the pattern
// kernel's segments past the head (head = true), or all of the validate
// kernel's segments.  0 = the block does not tile into segments (lane kernels).
int group_lanes(uint64_t bs, bool head = true) {
  if (bs < 2 * kSeg || bs % kSeg != 0) return 0;
  const uint64_t segs = bs / kSeg - (head ? 1 : 0);
  int g = 1;
  while (g < 64 && (uint64_t)g < segs) g <<= 1;
  return g;
}

template <template <int> class K, typename... A>
hipError_t launch_grouped(int g, uint64_t nblocks, hipStream_t s, A... args) {
  const uint64_t waves = (nblocks + (64 / g) - 1) / (64 / g);
  const uint32_t grid = grid_for(waves, 0, 64);
  switch (g) {
    case 1: return K<1>::go(grid, s, args...);
    case 2: return K<2>::go(grid, s, args...);
    case 4: return K<4>::go(grid, s, args...);
    case 8: return K<8>::go(grid, s, args...);
    case 16: return K<16>::go(grid, s, args...);
    case 32: return K<32>::go(grid, s, args...);
    default: return K<64>::go(grid, s, args...);
  }
}

template <int G>
struct ValidateK {
  static hipError_t go(uint32_t grid, hipStream_t s, const uint8_t* d, uint64_t n, uint64_t bs,
                       uint32_t* bad) {
    return launch(wave_validate_kernel<G>, grid, 64, 0, s, d, n, bs, bad);
  }
};
template <int G>
struct PatternK {
  static hipError_t go(uint32_t grid, hipStream_t s, uint8_t* d, uint64_t n, uint64_t bs,
                       uint64_t seed) {
    return launch(wave_pattern_kernel<G>, grid, 64, 0, s, d, n, bs, seed);
  }
};

}  // namespace

thread_local int g_validate_mode = 0;  // 0 auto, 1 lane, 2 grouped (xec_set_validate_kernel; per thread)

hipError_t launch_pattern(void* d_data, uint64_t nblocks, uint64_t bs, uint64_t seed,
                          hipStream_t s) {
  if (nblocks == 0) return hipSuccess;
  uint8_t* d = static_cast<uint8_t*>(d_data);
  const int g = group_lanes(bs);
  // The lane kernel wins once there are lanes enough for every block: its PCG
  // walk needs no jumps (config 4, 2 M blocks: 6.2 vs 14.6 ms, profiles/r02e).
  const bool grouped = g && (g_validate_mode == 2 || (g_validate_mode == 0 && nblocks < kLaneBlocks));
  if (grouped) return launch_grouped<PatternK>(g, nblocks, s, d, nblocks, bs, seed);
  return launch(serial_pattern_kernel, (uint32_t)((nblocks + 255) / 256), 256, 0, s, d, nblocks,
                bs, seed);
}

hipError_t launch_validate(const void* d_data, uint64_t nblocks, uint64_t bs, uint32_t* d_bad,
                           hipStream_t s) {
  const hipError_t z = hipMemsetAsync(d_bad, 0, sizeof(uint32_t), s);
  if (z != hipSuccess) return z;
  if (nblocks == 0) return hipSuccess;
  const uint8_t* d = static_cast<const uint8_t*>(d_data);
  const int g = group_lanes(bs, false);
  // Grouped lanes read each segment with 16-B loads a lane walks in order;
  // the lane kernel's strided walk loses even with 2 M blocks (profiles/r02e).
  if (g && g_validate_mode != 1) return launch_grouped<ValidateK>(g, nblocks, s, d, nblocks, bs, d_bad);
  return launch(serial_validate_kernel, (uint32_t)((nblocks + 255) / 256), 256, 0, s, d, nblocks,
                bs, d_bad);
}

// Loads this file's code object onto the current device (see xec_kernels.h).
hipError_t preload_validate() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&serial_validate_kernel));
}

}  // namespace xec
