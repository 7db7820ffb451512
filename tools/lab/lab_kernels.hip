// lab_kernels.hip -- experimental encode variants (NOT the product).
//
// Built into tools/lab/liblab.so by tools/lab/Makefile and driven by
// tools/lab/lab.py on the GPU box to decide what the product kernel in
// erasure-code-benchmark_amd/csrc/xec_kernels.hip should become.  Kept in a
// separate code object so lab instantiations cannot perturb the product's
// code generation (cdna_hip_programming.md §5.4 rule 19).
#include <hip/hip_runtime.h>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Dynamic LDS reserved per workgroup by the launches that honour it (residency
// cap, as the product's xec_set_occupancy); 0 = none.  Set by lab_set_ceiling_lds.
static uint32_t g_ceiling_lds = 0;
// Store policy of the decode diagnostics' default modes (2 = nt, as before;
// 16 = sc1, the product's decode policy).  Set by lab_set_dec_store_aux.
static int g_dec_store_aux = 2;

// cache-policy aux bits for buffer ops on gfx950: sc0 = 1, nt = 2, sc1 = 16
constexpr int GLOBAL_NT = -1;  // plain global_load/store with __builtin_nontemporal_*

struct Geo {
  uint64_t S, bs, k, m, tpb, total;
  int saux;  // decode diagnostics: result store policy (2 = nt, 16 = sc1)
};

template <int THREADS>
__device__ __forceinline__ void decompose(uint64_t t, int order, const Geo& g, uint64_t& c,
                                          uint64_t& j, uint64_t& chunk) {
  if (order == 1) {  // stripe fastest
    c = t % g.S;
    uint64_t r = t / g.S;
    j = r % g.m;
    chunk = r / g.m;
  } else {  // chunk fastest (product order)
    chunk = t % g.tpb;
    uint64_t r = t / g.tpb;
    j = r % g.m;
    c = r / g.m;
  }
}

template <int NM, int THREADS, int LAUX, int SAUX>
__device__ __forceinline__ void do_tile(const uint8_t* data, uint8_t* parity, uint64_t c, uint64_t j,
                                        uint64_t chunk, const Geo& g) {
  const uint64_t goff = (chunk * THREADS + threadIdx.x) * 16;
  if (goff >= g.bs) return;
  const uint8_t* base = data + (c * g.k + j) * g.bs;
  uint8_t* dst = parity + (c * g.m + j) * g.bs;
  const uint64_t stride = g.m * g.bs;
  u32x4 v[NM];
  if constexpr (LAUX == GLOBAL_NT) {
#pragma unroll
    for (int r = 0; r < NM; ++r)
      v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + r * stride + goff));
  } else {
    __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int r = 0; r < NM; ++r)
      v[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)goff, (uint32_t)(r * stride), LAUX);
  }
  u32x4 acc = v[0];
#pragma unroll
  for (int r = 1; r < NM; ++r) acc ^= v[r];
  if constexpr (SAUX == GLOBAL_NT) {
    __builtin_nontemporal_store(acc, reinterpret_cast<u32x4*>(dst + goff));
  } else {
    __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc((void*)dst, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(acc, ws, (uint32_t)goff, 0, SAUX);
  }
}

// order 0: chunk fastest, 1: stripe fastest, 2: chunk fastest with each XCD
// (blockIdx % 8) given a contiguous range of tiles.
template <int NM, int THREADS, int ORDER, int LAUX, int SAUX>
__global__ __launch_bounds__(THREADS) void enc_tile(const uint8_t* data, uint8_t* parity, Geo g) {
  uint64_t t = blockIdx.x;
  if (ORDER == 2) {
    const uint64_t per = (gridDim.x + 7) / 8;
    t = (blockIdx.x % 8) * per + blockIdx.x / 8;
  }
  if (t >= g.total) return;
  uint64_t c, j, chunk;
  decompose<THREADS>(t, ORDER == 1 ? 1 : 0, g, c, j, chunk);
  do_tile<NM, THREADS, LAUX, SAUX>(data, parity, c, j, chunk, g);
}

// persistent grid-stride with register double buffering: the next tile's
// loads are issued before the current tile is reduced and stored.
template <int NM, int THREADS>
__global__ __launch_bounds__(THREADS) void enc_persist_db(const uint8_t* data, uint8_t* parity, Geo g) {
  const uint64_t stride = g.m * g.bs;
  u32x4 cur[NM], nxt[NM];
  uint64_t t = blockIdx.x;
  auto load = [&](uint64_t tt, u32x4* v) {
    uint64_t c, j, chunk;
    decompose<THREADS>(tt, 0, g, c, j, chunk);
    const uint64_t goff = (chunk * THREADS + threadIdx.x) * 16;
    const uint8_t* base = data + (c * g.k + j) * g.bs;
#pragma unroll
    for (int r = 0; r < NM; ++r)
      v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + r * stride + goff));
  };
  if (t >= g.total) return;
  load(t, cur);
  for (; t < g.total; t += gridDim.x) {
    const uint64_t tn = t + gridDim.x;
    if (tn < g.total) load(tn, nxt);
    uint64_t c, j, chunk;
    decompose<THREADS>(t, 0, g, c, j, chunk);
    const uint64_t goff = (chunk * THREADS + threadIdx.x) * 16;
    u32x4 acc = cur[0];
#pragma unroll
    for (int r = 1; r < NM; ++r) acc ^= cur[r];
    __builtin_nontemporal_store(acc, reinterpret_cast<u32x4*>(parity + (c * g.m + j) * g.bs + goff));
#pragma unroll
    for (int r = 0; r < NM; ++r) cur[r] = nxt[r];
  }
}


// one-wave tiles of U granules per lane, register budget set by WPE (waves per
// SIMD the compiler must allow; lower = more VGPRs = more loads in flight)
template <int NM, int U, int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
void enc_wave(const uint8_t* data, uint8_t* parity, Geo g) {
  const uint64_t t = blockIdx.x;
  if (t >= g.total) return;
  uint64_t c, j, chunk;
  decompose<64>(t, 0, g, c, j, chunk);
  const uint64_t off = (chunk * 64 * U + threadIdx.x) * 16;
  const uint8_t* base = data + (c * g.k + j) * g.bs + off;
  uint8_t* dst = parity + (c * g.m + j) * g.bs + off;
  const uint64_t stride = g.m * g.bs;
  u32x4 v[NM][U];
#pragma unroll
  for (int r = 0; r < NM; ++r)
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[r][u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + r * stride + u * 1024));
#pragma unroll
  for (int u = 0; u < U; ++u) {
    u32x4 acc = v[0][u];
#pragma unroll
    for (int r = 1; r < NM; ++r) acc ^= v[r][u];
    __builtin_nontemporal_store(acc, reinterpret_cast<u32x4*>(dst + u * 1024));
  }
}


// ---- decode diagnostics (m = 1, one 1 KiB tile per one-wave workgroup) ----
// MODE 0: lost member from the bitmap row by lane loads + ballot (product)
// MODE 1: lost member from a per-stripe u8 table by one scalar load
// MODE 2: lost member computed as (7c) mod k -- no memory lookup (diagnostic)
// MODE 3: as 2 but the rebuilt block goes to a separate buffer (diagnostic)
// MODE 4: as 1 but with grid-stride and the next tile's table entry prefetched
// MODE 6: as 2, stripe-fastest tile order
// MODE 7: as 2, rebuilt block written to `out` at the same offset as in data (diagnostic)
// MODE 8: as 2, rebuilt block written to stripe (c + S/2) % S's lost slot (diagnostic)
// MODE 9: as 2, store with the default cache policy; MODE 10: store sc1 nt
// MODE 7 with `out` = the other buffer set's data (lab.py d12): another data buffer
// MODE 13: as 2, tiles in reverse order
// MODE 14/15: as 2, rebuilt chunk written to chunk + tpb/2 / chunk + 4 of the
// same lost block (diagnostic); MODE 16: to stripe c+1's lost slot; MODE 17:
// into the parity block (diagnostic)
template <int NM, int MODE>
__global__ __launch_bounds__(64) void dec_wave(uint8_t* data, const uint8_t* parity,
                                               const uint8_t* lookup, uint8_t* out, Geo g) {
  const uint32_t lane = threadIdx.x;
  const uint64_t stride = g.m * g.bs;
  for (uint64_t t0 = blockIdx.x; t0 < g.total; t0 += gridDim.x) {
    const uint64_t t = MODE == 13 ? g.total - 1 - t0 : t0;
    uint64_t c, j, chunk;
    decompose<64>(t, MODE == 6 ? 1 : 0, g, c, j, chunk);
    int lost;
    if (MODE == 0) {
      const uint8_t* row = lookup + c * (g.k + g.m) + j;
      const bool z = lane < NM && row[(uint64_t)lane * g.m] == 0;
      const uint64_t mask = __ballot(z);
      lost = mask ? __builtin_ctzll(mask) : -1;
    } else if (MODE == 11) {
      typedef const uint32_t __attribute__((address_space(4))) cu32;
      const uint64_t rowpos = c * (g.k + g.m) + j;
      lost = -1;
#pragma unroll
      for (int r = NM - 1; r >= 0; --r) {
        const uint64_t pos = rowpos + (uint64_t)r * g.m;
        const uint32_t w = *(cu32*)(lookup + (pos & ~3ull));
        if (((w >> (8 * (pos & 3))) & 0xffu) == 0) lost = r;
      }
    } else if (MODE == 1 || MODE == 4) {
      lost = (int)(int8_t)lookup[c * g.m + j];
    } else {
      lost = (int)((7 * c) % g.k);
    }
    lost = __builtin_amdgcn_readfirstlane(lost);
    if (lost < 0) continue;
    const uint64_t off = (chunk * 64 + lane) * 16;
    const uint8_t* base = data + (c * g.k + j) * g.bs;
    const uint8_t* par = parity + (c * g.m + j) * g.bs;
    u32x4 v[NM];
#pragma unroll
    for (int r = 0; r < NM; ++r)
      v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>((r == lost ? par : base + r * stride) + off));
    u32x4 acc = v[0];
#pragma unroll
    for (int r = 1; r < NM; ++r) acc ^= v[r];
    uint8_t* dst = data + (c * g.k + j) * g.bs + lost * stride;
    if (MODE == 3) dst = out + c * g.bs;
    if (MODE == 7) dst = out + (c * g.k + j) * g.bs + lost * stride;
    if (MODE == 14) dst = data + (c * g.k + j) * g.bs + lost * stride + ((chunk + g.tpb / 2) % g.tpb) * 1024 - chunk * 1024;
    if (MODE == 15) dst = data + (c * g.k + j) * g.bs + lost * stride + ((chunk + 4) % g.tpb) * 1024 - chunk * 1024;
    if (MODE == 16) {
      const uint64_t c2 = (c + 1) % g.S;
      dst = data + (c2 * g.k + j) * g.bs + ((7 * c2) % g.k) * stride;
    }
    if (MODE == 17) dst = const_cast<uint8_t*>(parity) + (c * g.m + j) * g.bs;
    if (MODE == 8) {
      const uint64_t c2 = (c + g.S / 2) % g.S;
      dst = data + (c2 * g.k + j) * g.bs + ((7 * c2) % g.k) * stride;
    }
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000);
    if (MODE == 9) __builtin_amdgcn_raw_buffer_store_b128(acc, rs, (uint32_t)off, 0, 0);
    else if (MODE == 10) __builtin_amdgcn_raw_buffer_store_b128(acc, rs, (uint32_t)off, 0, 0x12);
    else if (g.saux == 16) __builtin_amdgcn_raw_buffer_store_b128(acc, rs, (uint32_t)off, 0, 16);
    else __builtin_amdgcn_raw_buffer_store_b128(acc, rs, (uint32_t)off, 0, 2);
  }
}


// ---- bandwidth ceilings on the same access pattern (diagnostics) ----------
// R: the encode's 16 loads per lane, no store (kept alive by an impossible
// compare); W: the encode's store stream alone; C: 1 load + 1 store (copy).
template <int MODE>
__global__ __launch_bounds__(64) void ceiling(const uint8_t* data, uint8_t* parity, Geo g) {
  const uint64_t t = blockIdx.x;
  if (t >= g.total) return;
  uint64_t c, j, chunk;
  decompose<64>(t, 0, g, c, j, chunk);
  const uint64_t off = (chunk * 64 + threadIdx.x) * 16;
  const uint8_t* base = data + (c * g.k + j) * g.bs + off;
  uint8_t* dst = parity + (c * g.m + j) * g.bs;
  const uint64_t stride = g.m * g.bs;
  u32x4 acc = {0u, 0u, 0u, 0u};
  if (MODE == 0) {
    u32x4 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + r * stride));
#pragma unroll
    for (int r = 0; r < 16; ++r) acc ^= v[r];
    if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u && acc.z == 0xF39CC060u && acc.w == 0x5CEDC834u) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b128(acc, rs, (uint32_t)off, 0, 2);
    }
  } else {
    if (MODE == 2) acc = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base));
    else acc.x = (uint32_t)t;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(acc, rs, (uint32_t)off, 0, 2);
  }
}


// read-only ceiling with T-thread workgroups: each workgroup reads T*16 bytes
// contiguous of each of the 16 class members (tile of T*16 bytes).
template <int T>
__global__ __launch_bounds__(T) void ceiling_read_wg(const uint8_t* data, uint8_t* parity, Geo g) {
  const uint64_t tpb = g.bs / (T * 16);
  const uint64_t t = blockIdx.x;
  if (t >= g.S * tpb) return;
  const uint64_t c = t / tpb, chunk = t % tpb;
  const uint8_t* base = data + c * g.k * g.bs + chunk * T * 16 + threadIdx.x * 16;
  u32x4 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + r * g.bs));
  u32x4 acc = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int r = 0; r < 16; ++r) acc ^= v[r];
  if (acc.x == 0x9E3779B9u && acc.y == 0x7F4A7C15u && acc.z == 0xF39CC060u && acc.w == 0x5CEDC834u)
    parity[0] = 1;
}

// write-only bursts: each one-wave workgroup stores W KiB contiguous (W
// 16-byte stores per lane, 1 KiB apart) with cache policy AUX.
template <int W, int AUX>
__global__ __launch_bounds__(64) void wburst(uint8_t* out, uint64_t total_bytes) {
  const uint64_t base = (uint64_t)blockIdx.x * W * 1024;
  if (base >= total_bytes) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + base, 0, 0x7fffffff, 0x00020000);
  u32x4 v = {(uint32_t)blockIdx.x, threadIdx.x, 0x9E3779B9u, 0x7F4A7C15u};
#pragma unroll
  for (int i = 0; i < W; ++i)
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, (uint32_t)(i * 1024 + threadIdx.x * 16), 0, AUX);
}

// write-only, 1 KiB per one-wave workgroup, but workgroup b writes chunk
// remap(b): the GRP consecutive chunks of each group go to workgroups b with the
// same b % 8 (observed: same XCD), so one XCD writes GRP KiB contiguous.
template <int GRP, int AUX>
__global__ __launch_bounds__(64) void wburst_xcd(uint8_t* out, uint64_t total_bytes) {
  const uint64_t b = blockIdx.x;
  const uint64_t g = b / (8 * GRP), x = b % 8, slot = (b / 8) % GRP;
  const uint64_t chunk = g * 8 * GRP + x * GRP + slot;
  const uint64_t base = chunk * 1024;
  if (base >= total_bytes) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + base, 0, 0x7fffffff, 0x00020000);
  u32x4 v = {(uint32_t)b, threadIdx.x, 0x9E3779B9u, 0x7F4A7C15u};
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, (uint32_t)(threadIdx.x * 16), 0, AUX);
}

// write-only, T-thread workgroups, each lane one 16-byte store: T*16 bytes
// contiguous per workgroup.
template <int T>
__global__ __launch_bounds__(T) void wburst_wg(uint8_t* out, uint64_t total_bytes) {
  const uint64_t base = (uint64_t)blockIdx.x * T * 16;
  if (base >= total_bytes) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out + base, 0, 0x7fffffff, 0x00020000);
  u32x4 v = {(uint32_t)blockIdx.x, threadIdx.x, 0x9E3779B9u, 0x7F4A7C15u};
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, (uint32_t)(threadIdx.x * 16), 0, 2);
}

// write-only, scattered: nblk blocks of blk bytes, block b at byte b*stride;
// one-wave workgroup per 1 KiB (the decode's rebuilt-block store shape).
template <int AUX>
__global__ __launch_bounds__(64) void wscatter(uint8_t* out, uint64_t blk, uint64_t stride,
                                               uint64_t nblk) {
  const uint64_t per = blk / 1024, t = blockIdx.x;
  if (t >= nblk * per) return;
  uint8_t* base = out + (t / per) * stride + (t % per) * 1024;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  u32x4 v = {(uint32_t)t, threadIdx.x, 0x9E3779B9u, 0x7F4A7C15u};
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, (uint32_t)(threadIdx.x * 16), 0, AUX);
}

// one-wave workgroups that process TPW ADJACENT tiles in sequence (tile
// b*TPW + i): the store of tile i overlaps the loads of tile i+1.
template <int NM, int TPW>
__global__ __launch_bounds__(64) void enc_seq(const uint8_t* data, uint8_t* parity, Geo g) {
  const uint64_t stride = g.m * g.bs;
  for (int i = 0; i < TPW; ++i) {
    const uint64_t t = (uint64_t)blockIdx.x * TPW + i;
    if (t >= g.total) return;
    uint64_t c, j, chunk;
    decompose<64>(t, 0, g, c, j, chunk);
    const uint64_t off = (chunk * 64 + threadIdx.x) * 16;
    const uint8_t* base = data + (c * g.k + j) * g.bs + off;
    u32x4 v[NM];
#pragma unroll
    for (int r = 0; r < NM; ++r)
      v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + r * stride));
    u32x4 acc = v[0];
#pragma unroll
    for (int r = 1; r < NM; ++r) acc ^= v[r];
    uint8_t* dst = parity + (c * g.m + j) * g.bs;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(acc, rs, (uint32_t)off, 0, 2);
  }
}

// LDS staging (the north star's suggested shape): four waves each reduce four
// of the 16 members of a 1 KiB column, stage the partial in LDS, and wave 0
// combines the four partials and stores.
__global__ __launch_bounds__(256) void enc_lds(const uint8_t* data, uint8_t* parity, Geo g) {
  __shared__ u32x4 part[4][64];
  const uint64_t t = blockIdx.x;
  if (t >= g.total) return;
  uint64_t c, j, chunk;
  decompose<64>(t, 0, g, c, j, chunk);
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t off = (chunk * 64 + lane) * 16;
  const uint8_t* base = data + (c * g.k + j) * g.bs + off;
  const uint64_t stride = g.m * g.bs;
  u32x4 v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
    v[r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (w * 4 + r) * stride));
  part[w][lane] = v[0] ^ v[1] ^ v[2] ^ v[3];
  __syncthreads();
  if (w == 0) {
    const u32x4 acc = part[0][lane] ^ part[1][lane] ^ part[2][lane] ^ part[3][lane];
    uint8_t* dst = parity + (c * g.m + j) * g.bs;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(acc, rs, (uint32_t)off, 0, 2);
  }
}

// Wavefront shuffle reduction (member-split across lanes): each load
// instruction covers 8 members x 128 B (8 lanes per member), two cover the
// 16 members of a 128 B column; after XOR-ing the two, the 8 member groups are
// folded with lane-xor shuffles 8/16/32 and lanes 0-7 store 128 B.  Eight
// such columns make the 1 KiB tile; all 16 loads per lane are in flight.
__global__ __launch_bounds__(64) void enc_shfl(const uint8_t* data, uint8_t* parity, Geo g) {
  const uint64_t t = blockIdx.x;
  if (t >= g.total) return;
  uint64_t c, j, chunk;
  decompose<64>(t, 0, g, c, j, chunk);
  const uint32_t lane = threadIdx.x, sub = lane & 7, grp = lane >> 3;
  const uint64_t stride = g.m * g.bs;
  const uint8_t* base = data + (c * g.k + j) * g.bs + chunk * 1024 + sub * 16;
  u32x4 a[8], b[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    a[s] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + grp * stride + s * 128));
    b[s] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (grp + 8) * stride + s * 128));
  }
  uint8_t* dst = parity + (c * g.m + j) * g.bs;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    u32x4 x = a[s] ^ b[s];
#pragma unroll
    for (int mask = 8; mask < 64; mask <<= 1) {
      x.x ^= (uint32_t)__shfl_xor((int)x.x, mask, 64);
      x.y ^= (uint32_t)__shfl_xor((int)x.y, mask, 64);
      x.z ^= (uint32_t)__shfl_xor((int)x.z, mask, 64);
      x.w ^= (uint32_t)__shfl_xor((int)x.w, mask, 64);
    }
    if (grp == 0)
      __builtin_amdgcn_raw_buffer_store_b128(x, rs, (uint32_t)(chunk * 1024 + s * 128 + sub * 16), 0, 2);
  }
}

// Grouped multi-granule tiles: each lane owns UU granules 1 KiB apart (a
// UU KiB column per wave), members are processed G at a time (G*UU loads in
// flight), so each member is read as UU KiB contiguous per wave while the
// register budget stays at full occupancy.
template <int NM, int G, int UU>
__global__ __launch_bounds__(64) void enc_group_impl(const uint8_t* data, uint8_t* parity, Geo g) {
  const uint64_t tpb = g.tpb / UU;  // g.tpb counts 1 KiB tiles
  const uint64_t t = blockIdx.x;
  if (t >= g.S * g.m * tpb) return;
  const uint64_t chunk = t % tpb, cj = t / tpb, j = cj % g.m, c = cj / g.m;
  const uint64_t stride = g.m * g.bs;
  const uint8_t* base = data + (c * g.k + j) * g.bs + chunk * UU * 1024 + threadIdx.x * 16;
  u32x4 acc[UU];
#pragma unroll
  for (int u = 0; u < UU; ++u) acc[u] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
  for (int r0 = 0; r0 < NM; r0 += G) {
    u32x4 v[G][UU];
#pragma unroll
    for (int r = 0; r < G; ++r)
#pragma unroll
      for (int u = 0; u < UU; ++u)
        v[r][u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (r0 + r) * stride + u * 1024));
#pragma unroll
    for (int r = 0; r < G; ++r)
#pragma unroll
      for (int u = 0; u < UU; ++u) acc[u] ^= v[r][u];
  }
  uint8_t* dst = parity + (c * g.m + j) * g.bs;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int u = 0; u < UU; ++u)
    __builtin_amdgcn_raw_buffer_store_b128(acc[u], rs, (uint32_t)(chunk * UU * 1024 + u * 1024 + threadIdx.x * 16), 0, 2);
}

namespace {
template <int THREADS>
Geo geo(uint64_t S, uint64_t bs, uint64_t k, uint64_t m) {
  Geo g{S, bs, k, m, 0, 0, 2};
  g.tpb = (bs / 16 + THREADS - 1) / THREADS;
  g.total = S * m * g.tpb;
  return g;
}
template <int NM, int THREADS, int ORDER, int LAUX, int SAUX>
int launch(const void* d, void* p, uint64_t S, uint64_t bs, uint64_t k, uint64_t m, hipStream_t s) {
  Geo g = geo<THREADS>(S, bs, k, m);
  uint64_t grid = ORDER == 2 ? (g.total + 7) / 8 * 8 : g.total;
  enc_tile<NM, THREADS, ORDER, LAUX, SAUX><<<(uint32_t)grid, THREADS, 0, s>>>(
      static_cast<const uint8_t*>(d), static_cast<uint8_t*>(p), g);
  return hipGetLastError() == hipSuccess ? 0 : 6;
}
template <int NM, int U, int WPE>
int launch_wave(const void* d, void* p, uint64_t S, uint64_t bs, uint64_t k, uint64_t m, hipStream_t s) {
  Geo g = geo<64 * U>(S, bs, k, m);
  enc_wave<NM, U, WPE><<<(uint32_t)g.total, 64, 0, s>>>(static_cast<const uint8_t*>(d),
                                                       static_cast<uint8_t*>(p), g);
  return hipGetLastError() == hipSuccess ? 0 : 6;
}
template <int MODE>
int launch_dec(void* d, const void* p, const void* lookup, void* out, uint64_t S, uint64_t bs,
               uint64_t k, uint64_t m, uint32_t grid, hipStream_t s) {
  Geo g = geo<64>(S, bs, k, m);
  g.saux = g_dec_store_aux;
  dec_wave<16, MODE><<<grid ? grid : (uint32_t)g.total, 64, g_ceiling_lds, s>>>(
      static_cast<uint8_t*>(d), static_cast<const uint8_t*>(p), static_cast<const uint8_t*>(lookup),
      static_cast<uint8_t*>(out), g);
  return hipGetLastError() == hipSuccess ? 0 : 6;
}
template <int NM, int TPW>
int launch_seq(const void* d, void* p, uint64_t S, uint64_t bs, uint64_t k, uint64_t m, hipStream_t s) {
  Geo g = geo<64>(S, bs, k, m);
  enc_seq<NM, TPW><<<(uint32_t)((g.total + TPW - 1) / TPW), 64, 0, s>>>(
      static_cast<const uint8_t*>(d), static_cast<uint8_t*>(p), g);
  return hipGetLastError() == hipSuccess ? 0 : 6;
}
template <int NM, int G, int UU>
int launch_group(const void* d, void* p, uint64_t S, uint64_t bs, uint64_t k, uint64_t m, hipStream_t s) {
  if (bs % (UU * 1024)) return 1;
  Geo g = geo<64>(S, bs, k, m);
  static_assert(NM % G == 0, "G must divide the member count");
  enc_group_impl<NM, G, UU><<<(uint32_t)(S * m * (g.tpb / UU)), 64, g_ceiling_lds, s>>>(static_cast<const uint8_t*>(d),
                                                                     static_cast<uint8_t*>(p), g);
  return hipGetLastError() == hipSuccess ? 0 : 6;
}
template <int NM, int THREADS>
int launch_db(const void* d, void* p, uint64_t S, uint64_t bs, uint64_t k, uint64_t m, uint32_t grid,
              hipStream_t s) {
  Geo g = geo<THREADS>(S, bs, k, m);
  enc_persist_db<NM, THREADS><<<grid, THREADS, 0, s>>>(static_cast<const uint8_t*>(d),
                                                       static_cast<uint8_t*>(p), g);
  return hipGetLastError() == hipSuccess ? 0 : 6;
}
}  // namespace

extern "C" {

const char* lab_variant_name(int v) {
  static const char* names[] = {
      "A_glob_nt_256",     "B_buf_nt_nt_256",   "C_buf_ntsc1_nt_256", "D_buf_all_all_256",
      "E_buf_def_nt_256",  "F_stripe_first_nt", "G_xcd_contig_nt",    "H_glob_nt_512",
      "I_glob_nt_1024",    "J_glob_nt_64",      "K_persist_db_2048",  "L_persist_db_1024",
      "M_buf_sc1_nt_256",  "N_persist_db_4096", "O_buf_nt_sc1nt_256", "P_wave_u1_w8",
      "Q_wave_u1_w7",      "R_wave_u1_w6",      "S_wave_u1_w4",       "T_wave_u2_w4",
      "U_wave_u2_w5",      "V_wave_u2_w3",      "W_wave_u1_w5",       "X_seq_tpw1",
      "Y_seq_tpw2",        "Z_seq_tpw4",        "AA_lds_stage_256",   "AB_shfl_8x128_64",
      "AC_xcd_contig_64",  "AD_chunk_fast_64",  "AE_group_g4_u4",     "AF_group_g2_u4",
      "AG_group_g8_u2",    "AH_group_g4_u2",    "AI_group_g16_u1"};
  return (v >= 0 && v < (int)(sizeof names / sizeof *names)) ? names[v] : nullptr;
}

const char* lab_dec_name(int v) {
  static const char* names[] = {"d0_ballot", "d1_table", "d2_computed", "d3_computed_sepout",
                                "d4_table_gs8192", "d5_ballot_gs8192", "d6_stripe_first",
                                "d7_out_same_offset", "d8_far_stripe", "d9_store_default",
                                "d10_store_sc1nt", "d11_scalar_lookup", "d12_other_set_data",
                                "d13_reverse_order", "d14_chunk_half_shift", "d15_chunk_4k_shift",
                                "d16_next_stripe", "d17_into_parity"};
  return (v >= 0 && v < 18) ? names[v] : nullptr;
}

void lab_set_ceiling_lds(uint32_t bytes) { g_ceiling_lds = bytes; }
void lab_set_dec_store_aux(int aux) { g_dec_store_aux = aux; }

// Bandwidth ceilings on the encode's geometry (k = 16, m = 1): 0 read-only
// (bytes: S*k*bs), 1 write-only (S*bs), 2 copy of member 0 (2*S*bs).
int lab_ceiling(int mode, const void* d, void* p, uint64_t S, uint64_t bs, uint64_t k, uint64_t m,
                hipStream_t s) {
  Geo g = geo<64>(S, bs, k, m);
  const uint8_t* dd = static_cast<const uint8_t*>(d);
  uint8_t* pp = static_cast<uint8_t*>(p);
  const uint32_t lds = g_ceiling_lds;
  if (mode == 3) {
    ceiling_read_wg<256><<<(uint32_t)(S * (bs / 4096)), 256, lds, s>>>(dd, pp, g);
    return hipGetLastError() == hipSuccess ? 0 : 6;
  }
  if (mode == 4) {
    ceiling_read_wg<128><<<(uint32_t)(S * (bs / 2048)), 128, lds, s>>>(dd, pp, g);
    return hipGetLastError() == hipSuccess ? 0 : 6;
  }
  if (mode == 0) ceiling<0><<<(uint32_t)g.total, 64, lds, s>>>(dd, pp, g);
  else if (mode == 1) ceiling<1><<<(uint32_t)g.total, 64, lds, s>>>(dd, pp, g);
  else ceiling<2><<<(uint32_t)g.total, 64, lds, s>>>(dd, pp, g);
  return hipGetLastError() == hipSuccess ? 0 : 6;
}

// Write-only burst ceilings over `bytes` of `out`: variant 0..5 =
// (W, policy) in {1, 4, 16} KiB x {nt, sc1}.
int lab_wburst(int v, void* out, uint64_t bytes, hipStream_t s) {
  uint8_t* o = static_cast<uint8_t*>(out);
  const uint32_t lds = g_ceiling_lds;
  auto grid = [&](int w) { return (uint32_t)(bytes / (w * 1024ull)); };
  switch (v) {
    case 0: wburst<1, 2><<<grid(1), 64, lds, s>>>(o, bytes); break;
    case 1: wburst<4, 2><<<grid(4), 64, lds, s>>>(o, bytes); break;
    case 2: wburst<16, 2><<<grid(16), 64, lds, s>>>(o, bytes); break;
    case 3: wburst<1, 16><<<grid(1), 64, lds, s>>>(o, bytes); break;
    case 4: wburst<4, 16><<<grid(4), 64, lds, s>>>(o, bytes); break;
    case 5: wburst<16, 16><<<grid(16), 64, lds, s>>>(o, bytes); break;
    case 6: wburst_wg<256><<<grid(4), 256, lds, s>>>(o, bytes); break;
    case 7: wburst_xcd<4, 2><<<grid(1), 64, lds, s>>>(o, bytes); break;
    case 8: wburst<2, 2><<<grid(2), 64, lds, s>>>(o, bytes); break;
    case 9: wburst<8, 2><<<grid(8), 64, lds, s>>>(o, bytes); break;
    case 10: wburst_xcd<4, 16><<<grid(1), 64, lds, s>>>(o, bytes); break;
    case 11: wburst_xcd<2, 2><<<grid(1), 64, lds, s>>>(o, bytes); break;
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 6;
}

// Scattered write-only stream (wscatter): sc1 = 1 -> sc1 stores, else nt.
int lab_wscatter(int sc1, void* out, uint64_t blk, uint64_t stride, uint64_t nblk,
                 hipStream_t s) {
  if (blk < 1024 || blk % 1024 != 0 || stride < blk) return 1;
  const uint64_t n = nblk * (blk / 1024);
  if (n == 0 || n > 0x7fffffffu) return 1;
  uint8_t* o = static_cast<uint8_t*>(out);
  if (sc1) wscatter<16><<<(uint32_t)n, 64, g_ceiling_lds, s>>>(o, blk, stride, nblk);
  else wscatter<2><<<(uint32_t)n, 64, g_ceiling_lds, s>>>(o, blk, stride, nblk);
  return hipGetLastError() == hipSuccess ? 0 : 6;
}

// Decode diagnostics for k = 16, m = 1.  lookup = bitmap (d0, d5) or u8 table (d1, d4).
int lab_decode(int v, void* d, const void* p, const void* lookup, void* out, uint64_t S,
               uint64_t bs, uint64_t k, uint64_t m, hipStream_t s) {
  if (k != 16 || m != 1) return 3;
  switch (v) {
    case 0: return launch_dec<0>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 1: return launch_dec<1>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 2: return launch_dec<2>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 3: return launch_dec<3>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 4: return launch_dec<4>(d, p, lookup, out, S, bs, k, m, 8192, s);
    case 5: return launch_dec<0>(d, p, lookup, out, S, bs, k, m, 8192, s);
    case 6: return launch_dec<6>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 7: return launch_dec<7>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 8: return launch_dec<8>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 9: return launch_dec<9>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 10: return launch_dec<10>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 11: return launch_dec<11>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 12: return launch_dec<7>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 13: return launch_dec<13>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 14: return launch_dec<14>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 15: return launch_dec<15>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 16: return launch_dec<16>(d, p, lookup, out, S, bs, k, m, 0, s);
    case 17: return launch_dec<17>(d, p, lookup, out, S, bs, k, m, 0, s);
  }
  return 1;
}

// Encode for k/m == 16 (the benchmark shape).  Returns 0 or 6.
int lab_encode(int v, const void* d, void* p, uint64_t S, uint64_t bs, uint64_t k, uint64_t m,
               hipStream_t s) {
  if (k / m != 16) return 3;
  switch (v) {
    case 0: return launch<16, 256, 0, GLOBAL_NT, GLOBAL_NT>(d, p, S, bs, k, m, s);
    case 1: return launch<16, 256, 0, 2, 2>(d, p, S, bs, k, m, s);
    case 2: return launch<16, 256, 0, 0x12, 2>(d, p, S, bs, k, m, s);
    case 3: return launch<16, 256, 0, 0x13, 0x13>(d, p, S, bs, k, m, s);
    case 4: return launch<16, 256, 0, 0, 2>(d, p, S, bs, k, m, s);
    case 5: return launch<16, 256, 1, GLOBAL_NT, GLOBAL_NT>(d, p, S, bs, k, m, s);
    case 6: return launch<16, 256, 2, GLOBAL_NT, GLOBAL_NT>(d, p, S, bs, k, m, s);
    case 7: return launch<16, 512, 0, GLOBAL_NT, GLOBAL_NT>(d, p, S, bs, k, m, s);
    case 8: return launch<16, 1024, 0, GLOBAL_NT, GLOBAL_NT>(d, p, S, bs, k, m, s);
    case 9: return launch<16, 64, 0, GLOBAL_NT, GLOBAL_NT>(d, p, S, bs, k, m, s);
    case 10: return launch_db<16, 256>(d, p, S, bs, k, m, 2048, s);
    case 11: return launch_db<16, 256>(d, p, S, bs, k, m, 1024, s);
    case 12: return launch<16, 256, 0, 0x10, 2>(d, p, S, bs, k, m, s);
    case 13: return launch_db<16, 256>(d, p, S, bs, k, m, 4096, s);
    case 14: return launch<16, 256, 0, 2, 0x12>(d, p, S, bs, k, m, s);
    case 15: return launch_wave<16, 1, 8>(d, p, S, bs, k, m, s);
    case 16: return launch_wave<16, 1, 7>(d, p, S, bs, k, m, s);
    case 17: return launch_wave<16, 1, 6>(d, p, S, bs, k, m, s);
    case 18: return launch_wave<16, 1, 4>(d, p, S, bs, k, m, s);
    case 19: return launch_wave<16, 2, 4>(d, p, S, bs, k, m, s);
    case 20: return launch_wave<16, 2, 5>(d, p, S, bs, k, m, s);
    case 21: return launch_wave<16, 2, 3>(d, p, S, bs, k, m, s);
    case 22: return launch_wave<16, 1, 5>(d, p, S, bs, k, m, s);
    case 23: return launch_seq<16, 1>(d, p, S, bs, k, m, s);
    case 24: return launch_seq<16, 2>(d, p, S, bs, k, m, s);
    case 25: return launch_seq<16, 4>(d, p, S, bs, k, m, s);
    case 26: {
      if (bs % 1024) return 1;
      Geo g = geo<64>(S, bs, k, m);
      enc_lds<<<(uint32_t)g.total, 256, 0, s>>>(static_cast<const uint8_t*>(d), static_cast<uint8_t*>(p), g);
      return hipGetLastError() == hipSuccess ? 0 : 6;
    }
    case 27: {
      if (bs % 1024) return 1;
      Geo g = geo<64>(S, bs, k, m);
      enc_shfl<<<(uint32_t)g.total, 64, 0, s>>>(static_cast<const uint8_t*>(d), static_cast<uint8_t*>(p), g);
      return hipGetLastError() == hipSuccess ? 0 : 6;
    }
    case 28: return launch<16, 64, 2, GLOBAL_NT, 2>(d, p, S, bs, k, m, s);
    case 29: return launch<16, 64, 0, GLOBAL_NT, 2>(d, p, S, bs, k, m, s);
    case 30: return launch_group<16, 4, 4>(d, p, S, bs, k, m, s);
    case 31: return launch_group<16, 2, 4>(d, p, S, bs, k, m, s);
    case 32: return launch_group<16, 8, 2>(d, p, S, bs, k, m, s);
    case 33: return launch_group<16, 4, 2>(d, p, S, bs, k, m, s);
    case 34: return launch_group<16, 16, 1>(d, p, S, bs, k, m, s);
  }
  return 1;
}
}
