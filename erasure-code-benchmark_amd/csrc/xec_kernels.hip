// xec_kernels.hip -- CDNA4 (gfx950) kernels of the XOR-EC hot path.
//
// Written for MI355X from the reference's *behaviour*
// (src/xorec/xorec.cpp:24-111: parity class i % m, single-erasure rebuild),
// not from its CUDA kernels: there are no atomics, no memset pass and no
// 8-byte grid-stride loop here (cf. xorec_gpu_cmp.cu:119-208).
//
// Work unit ("tile"): one parity class j of one stripe c over a contiguous
// column range of T*U 16-byte granules (T = threads per workgroup, 64 or 256).
// A lane owns U granules of the column range and keeps every member of the
// class in flight at once:
//   encode: NM = k/m loads  (data blocks j, j+m, ...)      -> 1 parity store
//   decode: NM loads        (class members, lost one       -> 1 store into the
//                            replaced by the class parity)     lost data block
// so each wave-instruction is a fully coalesced 1 KiB global_load_dwordx4
// from one block and each lane has NM*U independent 16-byte loads in flight.
// The XOR reduction happens in registers; no LDS is needed because no byte is
// read twice and no cross-lane exchange is needed ("Why no LDS").
//
// Addresses are formed per load as (uniform block base) + r*stride + (lane
// offset) in 64-bit VGPR arithmetic.  Keeping an array of NM uniform member
// pointers instead costs ~2*NM SGPRs; above 80 SGPRs gfx950 admits one wave
// per SIMD fewer (MI355X_MICROARCH.md, Residency), which measured -5 % here.
//
// All byte offsets are 64-bit: the batch may exceed 4 GiB (cf. the 32-bit
// indices of xorec_gpu_cmp.cu:127-131).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "xec_kernels.h"

namespace xec {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// pointer into the constant address space: uniform loads through it become
// scalar (s_load) loads served by the scalar cache
typedef const uint32_t __attribute__((address_space(4)))* const_u32_as4;
typedef const int32_t __attribute__((address_space(4)))* const_i32_as4;

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
  if constexpr (NT) return __builtin_nontemporal_load(q);
  else return *q;
}

template <bool NT>
__device__ __forceinline__ void st16(uint8_t* p, u32x4 v) {
  u32x4* q = reinterpret_cast<u32x4*>(p);
  if constexpr (NT) __builtin_nontemporal_store(v, q);
  else *q = v;
}

// Cache policy of the result stores of the NT kernels (gfx950 buffer aux bits:
// sc0 = 1, nt = 2, sc1 = 16).  Encode stores parity `nt`.  Decode stores the
// rebuilt block `sc1`, which does not keep the line in the XCD's L2
// (MI355X_MICROARCH.md, stores of each flavour): the rebuilt line shares its
// L2 set with the same column of the blocks the tile is reading, and an
// in-place nt line left dirty there measured 3-6 % slower (config 3, config
// 2, 16+4, 32+1 x 64 KiB on two devices; bf0ca45:tools/archive/ab/patches/store_policy.py,
// profiles/r01r, r01s); for encode sc1 was -2..+3 %, so it stays nt.
constexpr int kEncodeStoreAux = 2;   // nt
constexpr int kDecodeStoreAux = 16;  // sc1

// Store 16 bytes at block + off.  With NT the store is a buffer store whose
// cache policy is an explicit operand (AUX): hipcc (ROCm 7.2) silently drops
// the !nontemporal of __builtin_nontemporal_store in the unrolled reduction
// below (the emitted global_store has no `nt`), which measured 5 % slower.
// tests/test_isa.py checks every NT kernel's stores carry their policy.
template <bool NT, int AUX>
__device__ __forceinline__ void st16_block(uint8_t* block, uint64_t off, u32x4 v) {
  if constexpr (NT) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(block, 0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, (uint32_t)off, 0, AUX);
  } else {
    st16<false>(block + off, v);
  }
}

// Decompose a tile index into (stripe c, class j, column chunk); chunks of
// one block are adjacent tile indices.
//
// kReverse note: both kernels hand workgroup b the tile total-1-b, i.e. walk
// the batch from its end.  In bench.py's encode/decode rotation that measured
// +1.1 % (encode +1.4 %, decode +0.8 %, three interleaved runs each,
// profiles/r01ae) and +2.1 / +1.2 % at config 3 in tools/ab (other shapes
// within +-0.8 %, profiles/r01ad); why is not known.
struct TileCoord {
  uint64_t c, j, chunk;
};

__device__ __forceinline__ TileCoord tile_coord(uint64_t t, const Geometry& g) {
  TileCoord tc;
  tc.chunk = t % g.tiles_per_block;
  const uint64_t cj = t / g.tiles_per_block;
  tc.j = cj % g.m;
  tc.c = cj / g.m;
  return tc;
}

// Column rotation (Geometry::rot, xec_set_rotation): stripe c's chunk q covers
// column chunk (q + c*rot) mod tiles_per_block.  A bijection on each block's
// chunks, so every byte is still read and written exactly once; it only moves
// which columns of concurrently read stripes are in flight together.  With
// one failed device -- the same shard lost in every stripe -- the stripes in
// flight read the same columns of blocks a power of two apart, which this HBM
// serves 10-20 % slower than a mix of offsets (tools/lab/read_probe.hip,
// profiles/r04b; DESIGN.md §3 *Which block is lost*).
__device__ __forceinline__ uint64_t rotated(uint64_t chunk, uint64_t c, const Geometry& g) {
  if (g.rot == 0) return chunk;
  const uint64_t q = chunk + (c * g.rot) % g.tiles_per_block;
  return q < g.tiles_per_block ? q : q - g.tiles_per_block;
}

// XOR-reduce the NM members of one class over this lane's U granules and
// store the result at dst.  Member r lives at base + r*stride, except member
// `subst`, whose bytes come from `sub` instead (decode: the class parity).
// `off` = this lane's byte offset of granule 0 in the block; granule u is
// off + u*T*16 and takes part only while inside the block (ragged tiles).
// SAUX = cache policy of the NT result store (kEncodeStoreAux / kDecodeStoreAux).
template <int NM, int U, bool NT, int T, int SAUX>
__device__ __forceinline__ void xor_members(const uint8_t* base, uint64_t stride,
                                            const uint8_t* sub, int subst, uint8_t* dst,
                                            uint64_t off, uint64_t bs, uint32_t nm_rt) {
  constexpr uint64_t kStep = (uint64_t)T * 16;
  if constexpr (NM > 0) {
    if (off + (U - 1) * kStep < bs) {  // whole tile inside the block: no predication
      u32x4 v[NM][U];
      // A running lane pointer (one 64-bit VGPR add per member) instead of NM
      // uniform member addresses, which the compiler would park in SGPRs.
      const uint8_t* p = base + off;
      const uint8_t* ps = sub + off;
#pragma unroll
      for (int r = 0; r < NM; ++r, p += stride) {
        const uint8_t* src = r == subst ? ps : p;
#pragma unroll
        for (int u = 0; u < U; ++u) v[r][u] = ld16<NT>(src + u * kStep);
      }
      // At 32+ members the compiler otherwise keeps a rolling window of ~11
      // loads in flight; with residency capped at one wave per SIMD
      // (xec_api.cpp auto_occupancy) all 32 in flight measured +4-6 %
      // (decode at config 4, encode at 32+1 x 64 KiB; tools/ab,
      // profiles/r01m).  At 16 members the window is faster (-2 %).
      if constexpr (NM >= 32) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        u32x4 acc = v[0][u];
#pragma unroll
        for (int r = 1; r < NM; ++r) acc ^= v[r][u];
        st16_block<NT, SAUX>(dst, off + u * kStep, acc);
      }
      return;
    }
  }
  // Ragged tail of a block, or a member count without a compiled unroll
  // (groups of 8 loads in flight per granule).
  const uint32_t nm = NM > 0 ? (uint32_t)NM : nm_rt;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t o = off + u * kStep;
    if (o >= bs) continue;
    u32x4 acc = {0u, 0u, 0u, 0u};
    uint32_t r = 0;
    for (; r + 8 <= nm; r += 8) {
      u32x4 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int rr = (int)(r + q);
        v[q] = ld16<NT>((rr == subst ? sub : base + (uint64_t)rr * stride) + o);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) acc ^= v[q];
    }
    for (; r < nm; ++r) acc ^= ld16<NT>(((int)r == subst ? sub : base + (uint64_t)r * stride) + o);
    st16_block<NT, SAUX>(dst, o, acc);
  }
}

// ---------------------------------------------------------------------------
// encode: parity[c][j] = XOR_{r < k/m} data[c][j + r*m]      (xorec.cpp:37-57)
// ---------------------------------------------------------------------------
template <int NM, int U, bool NT, int T>
__global__ __launch_bounds__(T) void encode_kernel(const uint8_t* __restrict__ data,
                                                   uint8_t* __restrict__ parity, Geometry g) {
  for (uint64_t t0 = blockIdx.x; t0 < g.total_tiles; t0 += gridDim.x) {
    // tiles are walked from the end of the batch (kReverse note above)
    const uint64_t t = g.total_tiles - 1 - t0;
    const TileCoord tc = tile_coord(t, g);
    const uint8_t* base = data + (tc.c * g.k + tc.j) * g.bs;
    uint8_t* dst = parity + (tc.c * g.m + tc.j) * g.bs;
    const uint64_t off = (rotated(tc.chunk, tc.c, g) * (uint64_t)(T * U) + threadIdx.x) * 16;
    xor_members<NM, U, NT, T, kEncodeStoreAux>(base, g.m * g.bs, nullptr, -1, dst, off, g.bs,
                                               (uint32_t)g.nm);
  }
}

// ---------------------------------------------------------------------------
// decode: every lost data block L (at most one per class, checked on the
// host) of class j = L % m is rebuilt as
//   data[c][L] = parity[c][j] ^ XOR_{r != L/m} data[c][j + r*m]  (xorec.cpp:79-108)
// A tile is (stripe c, column chunk) -- not per class -- so a workgroup only
// exists where there may be work: it scans the stripe's k data bitmap bytes
// with scalar loads (s_load_dword through the scalar cache; 4 bytes per load,
// exact zero-byte test in SALU) and rebuilds each lost block it finds.  With
// one erasure per stripe and m > 1 this launches m times fewer workgroups than
// a per-class tiling, of which m-1 in m would only have found nothing to do.
// Absolute addresses are used for the dword loads: the caller's scratch
// pointer need not be aligned, and an aligned dword never crosses a page.
// ---------------------------------------------------------------------------
template <int NM, int U, bool NT, int T>
__global__ __launch_bounds__(T) void decode_kernel(uint8_t* data, const uint8_t* __restrict__ parity,
                                                   const uint8_t* __restrict__ bitmap, Geometry g) {
  // xec_decode_device: the check kernel ran first on this stream; a failed
  // batch is left untouched (all-or-nothing, xorec_gpu_cmp.cu:75-81).
  if (g.gate != nullptr && *(const_i32_as4)g.gate != 0) return;
  const uint32_t nm = NM > 0 ? (uint32_t)NM : (uint32_t)g.nm;
  const uint32_t m = (uint32_t)g.m;
  const uint64_t stride = g.m * g.bs;
  for (uint64_t t0 = blockIdx.x; t0 < g.total_tiles; t0 += gridDim.x) {
    const uint64_t t = g.total_tiles - 1 - t0;  // from the end of the batch, as encode
    const uint64_t c = t / g.tiles_per_block;
    const uint64_t chunk = rotated(t % g.tiles_per_block, c, g);
    const uint64_t rowaddr = reinterpret_cast<uint64_t>(bitmap + c * (g.k + g.m));
    const uint64_t end = rowaddr + g.k;
    uint8_t* sdata = data + c * g.k * g.bs;
    const uint8_t* spar = parity + c * g.m * g.bs;
    const uint64_t off = (chunk * (uint64_t)(T * U) + threadIdx.x) * 16;
    for (uint64_t a = rowaddr & ~3ull; a < end; a += 4) {
      const uint32_t w = *(const_u32_as4)a;
      uint32_t z = ~(((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w) & 0x80808080u;  // zero bytes
      if (a < rowaddr) z &= 0xFFFFFFFFu << (8 * (uint32_t)(rowaddr - a));
      if (a + 4 > end) z &= 0xFFFFFFFFu >> (8 * (uint32_t)(a + 4 - end));
      while (z) {
        const uint32_t i = (uint32_t)(a - rowaddr) + ((uint32_t)__builtin_ctz(z) >> 3);
        z &= z - 1;
        const uint32_t j = i % m, r = i / m;  // class and member of lost block i
        uint8_t* base = sdata + (uint64_t)j * g.bs;
        xor_members<NM, U, NT, T, kDecodeStoreAux>(base, stride, spar + (uint64_t)j * g.bs,
                                                   (int)r, base + (uint64_t)r * stride, off,
                                                   g.bs, nm);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// decode, class tiles: the tile is encode's (stripe c, class j, column chunk).
// The workgroup reads its class's k/m data bitmap bytes (scalar dword loads,
// bytes j, j+m, ... of the stripe's row) and, if one of them is lost -- the
// host scan guarantees at most one -- rebuilds it with one class reduction,
// the encode's exact memory shape.  Chosen by the host when (nearly) every
// class of the batch lost a block (xec_api.cpp decode_tiling): then no tile is
// idle, and no tile runs several reductions back to back as the stripe tiles
// above do, whose rebuilt-block store sits in the same vmcnt queue as the
// next reduction's loads.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t sbyte(uint64_t addr) {
  const uint32_t w = *(const_u32_as4)(addr & ~3ull);
  return (w >> (8 * (uint32_t)(addr & 3))) & 0xFFu;
}

template <int NM, int U, bool NT, int T>
__global__ __launch_bounds__(T) void decode_class_kernel(uint8_t* data,
                                                         const uint8_t* __restrict__ parity,
                                                         const uint8_t* __restrict__ bitmap,
                                                         Geometry g) {
  if (g.gate != nullptr && *(const_i32_as4)g.gate != 0) return;
  const uint32_t nm = NM > 0 ? (uint32_t)NM : (uint32_t)g.nm;
  const uint64_t stride = g.m * g.bs;
  for (uint64_t t0 = blockIdx.x; t0 < g.total_tiles; t0 += gridDim.x) {
    const uint64_t t = g.total_tiles - 1 - t0;  // from the end of the batch, as encode
    const TileCoord tc = tile_coord(t, g);
    const uint64_t row = reinterpret_cast<uint64_t>(bitmap + tc.c * (g.k + g.m)) + tc.j;
    uint32_t lost = nm;
    for (uint32_t r = 0; r < nm; ++r)
      if (sbyte(row + (uint64_t)r * g.m) == 0) { lost = r; break; }
    if (lost == nm) continue;
    uint8_t* base = data + (tc.c * g.k + tc.j) * g.bs;
    const uint64_t off = (rotated(tc.chunk, tc.c, g) * (uint64_t)(T * U) + threadIdx.x) * 16;
    xor_members<NM, U, NT, T, kDecodeStoreAux>(base, stride, parity + (tc.c * g.m + tc.j) * g.bs,
                                               (int)lost, base + (uint64_t)lost * stride, off,
                                               g.bs, nm);
  }
}

// ---------------------------------------------------------------------------
// decode, work-list tiles: the host scan that xec_decode runs anyway lists the
// lost data blocks (c << 8 | i, xec_internal.h xec_work_item) and copies the
// list instead of the bitmap; a tile is (list entry, 1 KiB chunk) -- one class
// reduction, encode's memory shape -- so no tile is idle and none rebuilds
// several blocks back to back, whatever the losses' spread over the stripes.
// Tile t reads its entry with one scalar load.
// ---------------------------------------------------------------------------
template <int NM, int U, bool NT, int T>
__device__ __forceinline__ void rebuild_item(uint8_t* data, const uint8_t* __restrict__ parity,
                                             uint32_t item, uint64_t chunk, const Geometry& g) {
  const uint32_t nm = NM > 0 ? (uint32_t)NM : (uint32_t)g.nm;
  const uint32_t m = (uint32_t)g.m;
  const uint64_t stride = g.m * g.bs;
  const uint64_t c = item >> 8;
  const uint32_t i = item & 0xFFu;
  const uint32_t j = i % m, r = i / m;  // class and member of the lost block
  uint8_t* base = data + (c * g.k + j) * g.bs;
  const uint64_t off = (rotated(chunk, c, g) * (uint64_t)(T * U) + threadIdx.x) * 16;
  xor_members<NM, U, NT, T, kDecodeStoreAux>(base, stride, parity + (c * g.m + j) * g.bs, (int)r,
                                             base + (uint64_t)r * stride, off, g.bs, nm);
}

template <int NM, int U, bool NT, int T>
__global__ __launch_bounds__(T) void decode_list_kernel(uint8_t* data,
                                                        const uint8_t* __restrict__ parity,
                                                        const uint32_t* __restrict__ items,
                                                        Geometry g) {
  for (uint64_t t0 = blockIdx.x; t0 < g.total_tiles; t0 += gridDim.x) {
    const uint64_t t = g.total_tiles - 1 - t0;  // from the end of the batch, as encode
    const uint32_t item = *(const_u32_as4)(items + t / g.tiles_per_block);
    rebuild_item<NM, U, NT, T>(data, parity, item, t % g.tiles_per_block, g);
  }
}

// The same with the list in the kernel arguments (at most CAP entries, CAP
// one of 64 / 256 / 1024, xec_kernels.h arg_items_capacity; the item is a
// scalar load from the kernarg segment): small decodes then copy nothing to
// the device (a <= 8 KiB H2D copy runs as a blit kernel of its own,
// 3.7-4.4 us, profiles/r02o, r02l).
template <int NM, int U, bool NT, int T, uint32_t CAP>
__global__ __launch_bounds__(T) void decode_arglist_kernel(uint8_t* data,
                                                           const uint8_t* __restrict__ parity,
                                                           Geometry g, ArgItems<CAP> items) {
  for (uint64_t t0 = blockIdx.x; t0 < g.total_tiles; t0 += gridDim.x) {
    const uint64_t t = g.total_tiles - 1 - t0;
    rebuild_item<NM, U, NT, T>(data, parity, items.v[t / g.tiles_per_block],
                               t % g.tiles_per_block, g);
  }
}

// Argument-mask tiles (small batches: S <= 1,024 stripes, k <= 32): the losses
// travel in the kernel arguments as one mask per stripe (bit i = data block i
// lost), so a small decode copies nothing to the device whatever its number
// of losses -- in a synchronous call the bitmap copy is a blit kernel of its
// own ahead of the decode (3.7-4.4 us, profiles/r02o), as long as the
// reference's 8 MiB kernels themselves.  Two tilings, as over the bitmap:
//  * by_class: encode's (stripe, class, chunk) tiles, as decode_class_kernel.
//    A class holds at most one lost data block (the host scan's
//    recoverability check), so the tile's block is the lowest set bit of the
//    stripe's mask within the class's positions j, j+m, j+2m, ...;
//  * otherwise (stripe, chunk) tiles, as decode_kernel: the tile rebuilds
//    every block its stripe's mask names, one class reduction after another
//    (few losses per stripe: class tiles would mostly idle).
template <int NM, int U, bool NT, int T, uint32_t CAP>
__global__ __launch_bounds__(T) void decode_argmask_kernel(uint8_t* data,
                                                           const uint8_t* __restrict__ parity,
                                                           Geometry g, uint32_t by_class,
                                                           ArgItems<CAP> masks) {
  const uint32_t nm = NM > 0 ? (uint32_t)NM : (uint32_t)g.nm;
  const uint32_t m = (uint32_t)g.m;
  uint32_t class0 = 0;  // class 0's data positions: bits 0, m, 2m, ... (k <= 32)
  for (uint32_t r = 0; r < nm; ++r) class0 |= 1u << (r * m);
  for (uint64_t t0 = blockIdx.x; t0 < g.total_tiles; t0 += gridDim.x) {
    const uint64_t t = g.total_tiles - 1 - t0;  // from the end of the batch, as encode
    if (by_class) {
      const TileCoord tc = tile_coord(t, g);
      const uint32_t lost = masks.v[tc.c] & (class0 << tc.j);
      if (lost == 0) continue;
      rebuild_item<NM, U, NT, T>(data, parity,
                                 ((uint32_t)tc.c << 8) | (uint32_t)__builtin_ctz(lost), tc.chunk,
                                 g);
    } else {
      const uint64_t c = t / g.tiles_per_block, chunk = t % g.tiles_per_block;
      for (uint32_t lost = masks.v[c]; lost != 0; lost &= lost - 1)
        rebuild_item<NM, U, NT, T>(data, parity,
                                   ((uint32_t)c << 8) | (uint32_t)__builtin_ctz(lost), chunk, g);
    }
  }
}

// The same with a list the device built (xec_decode_device_list): list[0] is
// the entry count scan_list_kernel left, entries from list[1].  The host
// never sees the count, so the launch is a fixed grid (xec_api.cpp: one
// workgroup per 8 possible tiles, between what the chip holds at once and
// 131,072), walking the count's tiles in grid strides; workgroups past the
// list's end return at once.  On sparse batches that is 2-4x faster than
// decode_kernel over every stripe, and on dense ones within 1-4 % of one
// workgroup per tile (profiles/r06n); handing the tiles out in order from
// per-XCD work-queue heads instead was no better (0-31 % behind, commit
// 6f8fb1e, profiles/r02af, r02ag, r02ah), so the walk stays simple.  The gate
// is the check's verdict, as in decode_kernel.
template <int NM, int U, bool NT, int T>
__global__ __launch_bounds__(T) void decode_devlist_kernel(uint8_t* data,
                                                           const uint8_t* __restrict__ parity,
                                                           const uint32_t* __restrict__ list,
                                                           Geometry g) {
  if (*(const_i32_as4)g.gate != 0) return;
  const uint64_t total = (uint64_t)*(const_u32_as4)list * g.tiles_per_block;
  const uint32_t* entries = list + kDevListHeader;
  for (uint64_t t0 = blockIdx.x; t0 < total; t0 += gridDim.x) {
    const uint64_t t = total - 1 - t0;  // from the end of the list, as the other kernels
    const uint32_t item = *(const_u32_as4)(entries + t / g.tiles_per_block);
    rebuild_item<NM, U, NT, T>(data, parity, item, t % g.tiles_per_block, g);
  }
}

// ---------------------------------------------------------------------------
// check + list (xec_decode_device_list): one thread per (stripe, class), as
// check_kernel, and a class that lost exactly one block, a data block, appends
// its work item (c << 8 | i, xec_internal.h) after the list header.  A wave
// reserves its entries with one atomicAdd on the count (ballot + popcount), so entries
// come out grouped by wave, roughly in stripe order; their order does not
// matter -- each entry is rebuilt on its own.  A recoverable batch has at most
// one entry per class, so S*m entries always fit; an unrecoverable one gates
// the decode off whatever the list holds.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void scan_list_kernel(const uint8_t* __restrict__ bitmap,
                                                       Geometry g, int32_t* status,
                                                       uint32_t* list) {
  const uint64_t items = g.S * g.m, row = g.k + g.m;
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t b = (uint64_t)blockIdx.x * 256; b < items; b += (uint64_t)gridDim.x * 256) {
    const uint64_t t = b + threadIdx.x;  // the loop is uniform per workgroup: ballot sees every lane
    bool has = false;
    uint32_t entry = 0;
    if (t < items) {
      const uint64_t c = t / g.m, j = t % g.m;
      const uint8_t* r = bitmap + c * row;
      uint32_t lost = r[g.k + j] == 0, li = 0;
      for (uint64_t i = j; i < g.k; i += g.m)
        if (r[i] == 0) {
          ++lost;
          li = (uint32_t)i;
        }
      if (lost > 1) atomicOr(status, 4 /* XEC_DECODE_FAILURE */);
      has = lost == 1 && r[g.k + j] != 0;
      entry = (uint32_t)(c << 8) | li;
    }
    const uint64_t mask = __ballot(has);
    if (mask == 0) continue;
    const uint32_t leader = (uint32_t)__ffsll((unsigned long long)mask) - 1;
    uint32_t pos = 0;
    if (lane == leader) pos = atomicAdd(list, (uint32_t)__popcll(mask));
    pos = __shfl(pos, (int)leader);
    if (has) list[kDevListHeader + pos + (uint32_t)__popcll(mask & ((1ull << lane) - 1))] = entry;
  }
}

// *status = 0 and the list's count = 0 in one launch, stream-ordered before
// the scan.
__global__ void reset_status_list_kernel(int32_t* status, uint32_t* list) {
  *status = 0;
  *list = 0u;
}

// ---------------------------------------------------------------------------
// check: one thread per (stripe, class); counts the class's lost blocks among
// its k/m data bytes and its parity byte (is_recoverable, xorec_utils.hpp:160-175).
// Failure is rare, so the atomic is off the common path.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void check_kernel(const uint8_t* __restrict__ bitmap, Geometry g,
                                                    int32_t* status) {
  const uint64_t items = g.S * g.m, row = g.k + g.m;
  for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < items;
       t += (uint64_t)gridDim.x * 256) {
    const uint64_t c = t / g.m, j = t % g.m;
    const uint8_t* r = bitmap + c * row;
    uint32_t lost = r[g.k + j] == 0;
    for (uint64_t i = j; i < g.k; i += g.m) lost += r[i] == 0;
    if (lost > 1) atomicOr(status, 4 /* XEC_DECODE_FAILURE */);
  }
}

// ---------------------------------------------------------------------------
// erase: zero every block whose bitmap byte is 0 (abstract_bm.cpp:20-39)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void erase_kernel(uint8_t* data, uint8_t* parity,
                                                    const uint8_t* __restrict__ bitmap, Geometry g) {
  const uint64_t tot = g.k + g.m;
  const uint64_t nblocks = g.S * tot;
  const u32x4 zero = {0u, 0u, 0u, 0u};
  for (uint64_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
    if (bitmap[b] != 0) continue;
    const uint64_t c = b / tot, i = b % tot;
    uint8_t* blk = i < g.k ? data + (c * g.k + i) * g.bs : parity + (c * g.m + (i - g.k)) * g.bs;
    for (uint64_t x = threadIdx.x * 16ull; x < g.bs; x += 256 * 16) st16<false>(blk + x, zero);
  }
}

// ---------------------------------------------------------------------------
// gather: the host pipeline's rebuilt small blocks into one contiguous run
// (csrc/xec_pipeline.cpp: one D2H copy instead of one per block)
// ---------------------------------------------------------------------------
template <uint32_t CAP>
__global__ __launch_bounds__(256) void gather_kernel(const uint8_t* __restrict__ data,
                                                     uint8_t* __restrict__ out, uint64_t k,
                                                     uint64_t bs, uint32_t n, ArgItems<CAP> items) {
  for (uint32_t g = blockIdx.x; g < n; g += gridDim.x) {
    const uint32_t item = items.v[g];
    const uint8_t* src = data + ((uint64_t)(item >> 8) * k + (item & 0xFFu)) * bs;
    uint8_t* dst = out + (uint64_t)g * bs;
    for (uint64_t x = threadIdx.x * 16ull; x < bs; x += 256 * 16) st16<false>(dst + x, ld16<true>(src + x));
  }
}

// ---------------------------------------------------------------------------
// fill: splitmix64 stream per stripe, state seed_base + c
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix_at(uint64_t seed, uint64_t n) {
  uint64_t z = seed + (n + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void fill_kernel(uint64_t* buf, uint64_t S, uint64_t words,
                                                   uint64_t seed_base) {
  for (uint64_t c = blockIdx.y; c < S; c += gridDim.y) {
    uint64_t* row = buf + c * words;
    const uint64_t seed = seed_base + c;
    for (uint64_t n = (uint64_t)blockIdx.x * 256 + threadIdx.x; n < words;
         n += (uint64_t)gridDim.x * 256)
      row[n] = splitmix_at(seed, n);
  }
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
namespace {

template <int NM, int U, bool NT, int T>
hipError_t launch_encode_t(const void* d, void* p, const Geometry& g, uint32_t grid,
                           uint32_t lds, hipStream_t s) {
  return launch_codec(encode_kernel<NM, U, NT, T>, grid, T, lds, s,
                      static_cast<const uint8_t*>(d), static_cast<uint8_t*>(p), g);
}

// The first n of h_items in an ArgItems<CAP>, the rest zero (the kernel never
// reads past n; zeroed so a launch's arguments depend on the list alone).
template <uint32_t CAP>
ArgItems<CAP> arg_items(const uint32_t* h_items, uint64_t n) {
  ArgItems<CAP> a;
  std::memcpy(a.v, h_items, n * sizeof(uint32_t));
  std::memset(a.v + n, 0, (CAP - n) * sizeof(uint32_t));
  return a;
}

struct ArgList {
  const uint32_t* items;  // host memory, read at launch
  uint64_t n;             // <= kArgItems
};

template <int NM, int U, bool NT, int T>
hipError_t launch_decode_t(void* d, const void* p, const uint8_t* bm, const Geometry& g,
                           int tiling, uint32_t grid, uint32_t lds, hipStream_t s,
                           const ArgList& al) {
  uint8_t* dd = static_cast<uint8_t*>(d);
  const uint8_t* pp = static_cast<const uint8_t*>(p);
  const uint32_t* list = reinterpret_cast<const uint32_t*>(bm);
  if (tiling == kDecodeDevListTiles)
    return launch_codec(decode_devlist_kernel<NM, U, NT, T>, grid, T, lds, s, dd, pp, list, g);
  if (tiling == kDecodeArgListTiles) {
    switch (arg_items_capacity(al.n)) {
      case 64:
        return launch_codec(decode_arglist_kernel<NM, U, NT, T, 64>, grid, T, lds, s, dd, pp, g,
                      arg_items<64>(al.items, al.n));
      case 256:
        return launch_codec(decode_arglist_kernel<NM, U, NT, T, 256>, grid, T, lds, s, dd, pp, g,
                      arg_items<256>(al.items, al.n));
      default:
        return launch_codec(decode_arglist_kernel<NM, U, NT, T, 1024>, grid, T, lds, s, dd, pp, g,
                      arg_items<1024>(al.items, al.n));
    }
  }
  if (tiling == kDecodeArgMaskTiles || tiling == kDecodeArgMaskStripeTiles) {
    const uint32_t by_class = tiling == kDecodeArgMaskTiles;
    switch (arg_items_capacity(al.n)) {
      case 64:
        return launch_codec(decode_argmask_kernel<NM, U, NT, T, 64>, grid, T, lds, s, dd, pp, g,
                            by_class, arg_items<64>(al.items, al.n));
      case 256:
        return launch_codec(decode_argmask_kernel<NM, U, NT, T, 256>, grid, T, lds, s, dd, pp, g,
                            by_class, arg_items<256>(al.items, al.n));
      default:
        return launch_codec(decode_argmask_kernel<NM, U, NT, T, 1024>, grid, T, lds, s, dd, pp, g,
                            by_class, arg_items<1024>(al.items, al.n));
    }
  }
  if (tiling == kDecodeListTiles)
    return launch_codec(decode_list_kernel<NM, U, NT, T>, grid, T, lds, s, dd, pp, list, g);
  if (tiling == kDecodeClassTiles)
    return launch_codec(decode_class_kernel<NM, U, NT, T>, grid, T, lds, s, dd, pp, bm, g);
  return launch_codec(decode_kernel<NM, U, NT, T>, grid, T, lds, s, dd, pp, bm, g);
}

// Member counts (k/m) compiled fully unrolled: those of the reference's sweep
// (bm_config.cpp:7-11) and BASELINE.json -- 1, 2, 4, 8, 16, 32; others run the
// generic loop (NM = 0).
#define XEC_NM_SWITCH(NMV, CALL)                  \
  switch (NMV) {                                  \
    case 1: { constexpr int NM = 1; CALL; }       \
    case 2: { constexpr int NM = 2; CALL; }       \
    case 4: { constexpr int NM = 4; CALL; }       \
    case 8: { constexpr int NM = 8; CALL; }       \
    case 16: { constexpr int NM = 16; CALL; }     \
    case 32: { constexpr int NM = 32; CALL; }     \
    default: { constexpr int NM = 0; CALL; }      \
  }

template <int U, bool NT, int T>
hipError_t enc_nm(const void* d, void* p, const Geometry& g, uint32_t grid, uint32_t lds,
                  hipStream_t s) {
  XEC_NM_SWITCH(g.nm, return (launch_encode_t<NM, U, NT, T>(d, p, g, grid, lds, s)))
}

template <int U, bool NT, int T>
hipError_t dec_nm(void* d, const void* p, const uint8_t* bm, const Geometry& g, int tiling,
                  uint32_t grid, uint32_t lds, hipStream_t s, const ArgList& a) {
  XEC_NM_SWITCH(g.nm,
                return (launch_decode_t<NM, U, NT, T>(d, p, bm, g, tiling, grid, lds, s, a)))
}

template <bool NT, int T>
hipError_t enc_u(const void* d, void* p, const Geometry& g, int unroll, uint32_t grid,
                 uint32_t lds, hipStream_t s) {
  return unroll == 2 ? enc_nm<2, NT, T>(d, p, g, grid, lds, s)
                     : enc_nm<1, NT, T>(d, p, g, grid, lds, s);
}

template <bool NT, int T>
hipError_t dec_u(void* d, const void* p, const uint8_t* bm, const Geometry& g, int tiling,
                 int unroll, uint32_t grid, uint32_t lds, hipStream_t s, const ArgList& a) {
  return unroll == 2 ? dec_nm<2, NT, T>(d, p, bm, g, tiling, grid, lds, s, a)
                     : dec_nm<1, NT, T>(d, p, bm, g, tiling, grid, lds, s, a);
}

}  // namespace

hipError_t launch_encode(const void* d_data, void* d_parity, const Geometry& g,
                         const LaunchShape& ls, hipStream_t s) {
  const uint32_t grid = grid_for(g.total_tiles, ls.max_grid, ls.threads);
  const uint32_t lds = ls.lds_bytes;
  if (ls.threads == 256)
    return ls.nt ? enc_u<true, 256>(d_data, d_parity, g, ls.unroll, grid, lds, s)
                 : enc_u<false, 256>(d_data, d_parity, g, ls.unroll, grid, lds, s);
  return ls.nt ? enc_u<true, 64>(d_data, d_parity, g, ls.unroll, grid, lds, s)
               : enc_u<false, 64>(d_data, d_parity, g, ls.unroll, grid, lds, s);
}

hipError_t launch_decode(void* d_data, const void* d_parity, const uint8_t* d_bitmap,
                         const Geometry& g_class, const LaunchShape& ls, int tiling,
                         hipStream_t s, uint64_t n_items, const uint32_t* h_items) {
  // stripe tiles (stripe, chunk): decode_kernel; class tiles (stripe, class,
  // chunk) = encode's tiling: decode_class_kernel (with m == 1 the two
  // coincide and the stripe kernel runs); list tiles (entry, chunk):
  // decode_list_kernel over the n_items entries d_bitmap holds, or
  // decode_arglist_kernel over h_items (<= kArgItems) passed by value;
  // device-built list: decode_devlist_kernel over the count d_bitmap[0]
  // holds (n_items = its upper bound, which only sizes the grid); argument
  // masks: decode_argmask_kernel over class (or stripe) tiles, h_items = S
  // stripe masks.
  Geometry g = g_class;
  if (tiling == kDecodeClassTiles && g.m <= 1) tiling = kDecodeStripeTiles;
  if (tiling == kDecodeStripeTiles || tiling == kDecodeArgMaskStripeTiles)
    g.total_tiles = g.S * g.tiles_per_block;
  if (tiling == kDecodeListTiles || tiling == kDecodeArgListTiles ||
      tiling == kDecodeDevListTiles)
    g.total_tiles = n_items * g.tiles_per_block;
  if (g.total_tiles == 0) return hipSuccess;
  if (tiling == kDecodeArgListTiles && (n_items > kArgItems || h_items == nullptr))
    return hipErrorInvalidValue;
  if ((tiling == kDecodeArgMaskTiles || tiling == kDecodeArgMaskStripeTiles) &&
      (n_items != g.S || n_items > kArgItems || g.k > kArgMaskMaxK || h_items == nullptr))
    return hipErrorInvalidValue;
  const ArgList a{h_items, n_items};
  const uint32_t grid = grid_for(g.total_tiles, ls.max_grid, ls.threads);
  const uint32_t lds = ls.lds_bytes;
  if (ls.threads == 256)
    return ls.nt
               ? dec_u<true, 256>(d_data, d_parity, d_bitmap, g, tiling, ls.unroll, grid, lds, s, a)
               : dec_u<false, 256>(d_data, d_parity, d_bitmap, g, tiling, ls.unroll, grid, lds, s,
                                   a);
  return ls.nt ? dec_u<true, 64>(d_data, d_parity, d_bitmap, g, tiling, ls.unroll, grid, lds, s, a)
               : dec_u<false, 64>(d_data, d_parity, d_bitmap, g, tiling, ls.unroll, grid, lds, s,
                                  a);
}

hipError_t launch_check(const uint8_t* d_bitmap, const Geometry& g, int32_t* d_status,
                        hipStream_t s) {
  const uint32_t grid = grid_for((g.S * g.m + 255) / 256, 8192, 256);
  return launch(check_kernel, grid, 256, 0, s, d_bitmap, g, d_status);
}

hipError_t launch_scan_list(const uint8_t* d_bitmap, const Geometry& g, int32_t* d_status,
                            uint32_t* d_list, hipStream_t s) {
  const hipError_t e = launch(reset_status_list_kernel, 1, 1, 0, s, d_status, d_list);
  if (e != hipSuccess) return e;
  const uint32_t grid = grid_for((g.S * g.m + 255) / 256, 8192, 256);
  return launch(scan_list_kernel, grid, 256, 0, s, d_bitmap, g, d_status, d_list);
}

hipError_t launch_erase(void* d_data, void* d_parity, const uint8_t* d_bitmap, const Geometry& g,
                        hipStream_t s) {
  const uint64_t nblocks = g.S * (g.k + g.m);
  const uint32_t grid = grid_for(nblocks, 65536, 256);
  return launch(erase_kernel, grid, 256, 0, s, static_cast<uint8_t*>(d_data),
                static_cast<uint8_t*>(d_parity), d_bitmap, g);
}

hipError_t launch_gather(const void* d_data, void* d_out, uint64_t k, uint64_t bs,
                         const uint32_t* h_items, uint64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (n > kArgItems || k == 0 || k > 256 || bs % 16 != 0 || h_items == nullptr)
    return hipErrorInvalidValue;
  const uint8_t* src = static_cast<const uint8_t*>(d_data);
  uint8_t* dst = static_cast<uint8_t*>(d_out);
  const uint32_t grid = grid_for(n, 0, 256);
  switch (arg_items_capacity(n)) {
    case 64:
      return launch(gather_kernel<64>, grid, 256, 0, s, src, dst, k, bs, (uint32_t)n,
                    arg_items<64>(h_items, n));
    case 256:
      return launch(gather_kernel<256>, grid, 256, 0, s, src, dst, k, bs, (uint32_t)n,
                    arg_items<256>(h_items, n));
    default:
      return launch(gather_kernel<1024>, grid, 256, 0, s, src, dst, k, bs, (uint32_t)n,
                    arg_items<1024>(h_items, n));
  }
}

hipError_t launch_fill(void* d_buf, uint64_t S, uint64_t words, uint64_t seed_base,
                       hipStream_t s) {
  uint64_t gx = (words + 255) / 256;
  if (gx > 1024) gx = 1024;
  const uint64_t gy = S < 65535 ? S : 65535;
  if (gx == 0 || gy == 0) return hipSuccess;
  return launch(fill_kernel, dim3((uint32_t)gx, (uint32_t)gy), 256, 0, s,
                static_cast<uint64_t*>(d_buf), S, words, seed_base);
}

// Test hook only (tests/host/error_preserve.cpp).  A user who finds it set
// is told once, on stderr, that every launch of the library will fail
// (a silent hook in the shipped library).
thread_local KernelEvents t_kernel_events;

bool fail_launch_for_test() {
  static const bool on = [] {
    const char* e = std::getenv("XEC_TEST_FAIL_LAUNCH");
    const bool set = e != nullptr && e[0] == '1';
    if (set)
      std::fprintf(stderr,
                   "xec: XEC_TEST_FAIL_LAUNCH=1 is set: a TEST hook -- every kernel launch of "
                   "libxec_hip.so will fail on purpose\n");
    return set;
  }();
  return on;
}

// Loads this file's code object onto the current device (see xec_kernels.h).
hipError_t preload_kernels() {
  hipFuncAttributes a;
  return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&fill_kernel));
}

}  // namespace xec
