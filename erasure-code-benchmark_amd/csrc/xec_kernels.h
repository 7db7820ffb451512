// xec_kernels.h -- internal interface between the C ABI (xec_api.cpp) and the
// gfx950 kernels (xec_kernels.hip).  Not part of the public boundary.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdint>

namespace xec {

// Batch geometry.  A tile is one class of one stripe over threads*unroll
// 16-byte granules of the block.
struct Geometry {
  uint64_t S;                // stripes
  uint64_t k, m, nm;         // data blocks, parity blocks, members per class (k/m)
  uint64_t bs;               // bytes per block
  uint64_t tiles_per_block;  // ceil(bs / (16 * threads * unroll))
  uint64_t total_tiles;      // S * m * tiles_per_block
  const int32_t* gate;       // decode only: skip all work if *gate != 0 (nullptr = no gate)
  uint64_t rot;              // column rotation: stripe c's chunk q covers column chunk
                             // (q + c*rot) mod tiles_per_block (0 = none; xec_set_rotation)
};

struct LaunchShape {
  int threads;        // workgroup size: 64 (one wave) or 256
  int unroll;         // granules per lane per class member: 1 or 2
  uint32_t max_grid;  // 0 = one workgroup per tile, else grid-stride over tiles
  bool nt;            // non-temporal loads/stores
  uint32_t lds_bytes; // LDS reserved per workgroup to cap residency (0 = none)
  uint32_t rot = 0;   // column rotation in tiles per stripe (Geometry::rot)
};

inline Geometry make_geometry(uint64_t S, uint64_t bs, uint64_t k, uint64_t m,
                              const LaunchShape& ls) {
  Geometry g;
  g.S = S;
  g.k = k;
  g.m = m;
  g.nm = k / m;
  g.bs = bs;
  const uint64_t tile_bytes = 16ull * (uint64_t)ls.threads * (uint64_t)ls.unroll;
  g.tiles_per_block = (bs + tile_bytes - 1) / tile_bytes;
  g.total_tiles = S * m * g.tiles_per_block;
  g.gate = nullptr;
  g.rot = g.tiles_per_block > 1 ? ls.rot % g.tiles_per_block : 0;
  return g;
}

// Workgroups for `work_items` tiles of a grid-stride kernel: one per tile up
// to max_grid (0 = no cap of the caller's) and never beyond what HIP accepts,
// gridDim.x * blockDim.x <= 2^32 - 1; the kernels' grid-stride loops cover the
// rest.
inline uint32_t grid_for(uint64_t work_items, uint32_t max_grid, uint32_t threads) {
  const uint64_t hw = 0xFFFFFFFFull / (threads ? threads : 1);
  const uint64_t cap = max_grid && max_grid < hw ? (uint64_t)max_grid : hw;
  const uint64_t grid = work_items < cap ? work_items : cap;
  return (uint32_t)(grid ? grid : 1);
}

// Test hook: XEC_TEST_FAIL_LAUNCH=1 in the environment (read once) makes every
// kernel launch of the library invalid (2048 threads per workgroup), so that a
// test sees the wrappers report a genuine launch failure while an error of the
// caller's with the same code is pending (tests/host/error_preserve.cpp).
bool fail_launch_for_test();

// xec_set_kernel_events: events the next codec kernel launch of this thread
// records from its own dispatch (hipExtLaunchKernel), then forgets.  Set by
// the ABI call, cleared when the codec call that follows returns
// (KernelEventsScope, xec_api.cpp), consumed by launch_codec below.
struct KernelEvents {
  hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local KernelEvents t_kernel_events;

template <typename T>
struct NoDeduce {
  using type = T;
};

// Launches `kernel` and returns THIS launch's status, from hipLaunchKernel
// itself.  The thread's pending error is neither read nor cleared: one the
// caller left unread stays theirs (a successful launch does not touch it,
// tools/lab/last_error_probe.hip, profiles/r05b), and a failed launch is
// reported whatever was pending before (comparing the pending
// error before and after took a failure with the caller's code for success).
template <typename... P>
hipError_t launch(void (*kernel)(P...), dim3 grid, dim3 block, uint32_t lds, hipStream_t s,
                  typename NoDeduce<P>::type... args) {
  void* argv[] = {static_cast<void*>(&args)...};
  if (fail_launch_for_test()) block = dim3(2048);
  return hipLaunchKernel(reinterpret_cast<const void*>(kernel), grid, block, argv, lds, s);
}

// The codec kernels (encode and every decode tiling) go through this: as
// launch(), but with the thread's pending kernel events, if any, recorded by
// the kernel's dispatch itself and then cleared.
template <typename... P>
hipError_t launch_codec(void (*kernel)(P...), dim3 grid, dim3 block, uint32_t lds, hipStream_t s,
                        typename NoDeduce<P>::type... args) {
  const KernelEvents ev = t_kernel_events;
  if (ev.start == nullptr && ev.stop == nullptr)
    return launch(kernel, grid, block, lds, s, args...);
  t_kernel_events = KernelEvents{};
  void* argv[] = {static_cast<void*>(&args)...};
  if (fail_launch_for_test()) block = dim3(2048);
  return hipExtLaunchKernel(reinterpret_cast<const void*>(kernel), grid, block, argv, lds, s,
                            ev.start, ev.stop, 0);
}

hipError_t launch_encode(const void* d_data, void* d_parity, const Geometry& g,
                         const LaunchShape& ls, hipStream_t s);
// Decode tilings.  Stripe: one tile per (stripe, chunk), d_bitmap = the batch
// bitmap.  Class: one per (stripe, class, chunk), d_bitmap = the bitmap.
// List: one per (work item, chunk), d_bitmap = n_items u32 work items
// (xec_internal.h xec_work_item), 4-byte aligned.
// ArgList: list tiles over up to kArgItems work items passed by value in the
// kernel arguments (h_items, host memory, read at launch): no copy at all.
// ArgMask (below): class or stripe tiles, the losses by value in the kernel
// arguments.
constexpr int kDecodeStripeTiles = 0;
constexpr int kDecodeClassTiles = 1;
constexpr int kDecodeListTiles = 2;
constexpr int kDecodeArgListTiles = 3;
// DevList: list tiles over a list the device built (launch_scan_list):
// d_bitmap = the u32 list, [0] = entry count, entries from [kDevListHeader];
// n_items = the most entries there can be (sizes the grid with ls.max_grid;
// g.gate must be set).
constexpr int kDecodeDevListTiles = 4;
constexpr uint32_t kDevListHeader = 1;  // u32 words before the first entry
// ArgMask: class tiles (stripe, class, chunk) over S <= kArgItems stripes whose
// losses travel in the kernel arguments as one mask per stripe (h_items[c] bit
// i = data block i lost; k <= kArgMaskMaxK), n_items = S: a small decode with
// any number of losses copies nothing to the device.  ArgMaskStripe: the same
// masks over stripe tiles (stripe, chunk).
constexpr int kDecodeArgMaskTiles = 5;
constexpr int kDecodeArgMaskStripeTiles = 6;
constexpr uint64_t kArgMaskMaxK = 32;
// The list travels in the kernel arguments, so a launch ships the whole array
// whatever the list's length: each kernel that takes one is compiled for three
// capacities and the launch picks the smallest that holds the list (VERDICT
// r05 item 4).  A kernel with 4 KiB of arguments costs 0.15-0.4 us more per
// synchronous call than the same kernel with 256 B (tools/latency,
// profiles/r06b): small, but free to avoid.
constexpr uint64_t kArgItems = 1024;  // the largest capacity
template <uint32_t N>
struct ArgItems {
  uint32_t v[N];
};
inline uint32_t arg_items_capacity(uint64_t n) { return n <= 64 ? 64 : n <= 256 ? 256 : 1024; }
hipError_t launch_decode(void* d_data, const void* d_parity, const uint8_t* d_bitmap,
                         const Geometry& g, const LaunchShape& ls, int tiling, hipStream_t s,
                         uint64_t n_items = 0, const uint32_t* h_items = nullptr);
// Device-side recoverability check (xorec_utils.hpp:160-175 over the batch):
// *d_status |= 4 if some class of some stripe lost two or more blocks.  The
// caller zeroes *d_status first (stream-ordered).
hipError_t launch_check(const uint8_t* d_bitmap, const Geometry& g, int32_t* d_status,
                        hipStream_t s);
// The same check, and the list of lost data blocks for kDecodeDevListTiles
// into d_list (header zeroed here with *d_status first; at most S*m entries).
hipError_t launch_scan_list(const uint8_t* d_bitmap, const Geometry& g, int32_t* d_status,
                            uint32_t* d_list, hipStream_t s);
hipError_t launch_erase(void* d_data, void* d_parity, const uint8_t* d_bitmap, const Geometry& g,
                        hipStream_t s);
hipError_t launch_fill(void* d_buf, uint64_t S, uint64_t words, uint64_t seed_base,
                       hipStream_t s);
// Gather (xec_pipeline's small-block decode): block i of stripe c of a chunk
// (item c << 8 | i, at most kArgItems items, k <= 256) is copied from
// d_data + (c*k + i)*bs to d_out + g*bs for the g-th item, so the chunk's
// rebuilt blocks leave in one D2H copy.  bs % 16 == 0.
hipError_t launch_gather(const void* d_data, void* d_out, uint64_t k, uint64_t bs,
                         const uint32_t* h_items, uint64_t n, hipStream_t s);
// xec_set_validate_kernel: 0 auto, 1 lane per block, 2 wave per block.
extern thread_local int g_validate_mode;
hipError_t launch_pattern(void* d_data, uint64_t nblocks, uint64_t bs, uint64_t seed,
                          hipStream_t s);
hipError_t launch_validate(const void* d_data, uint64_t nblocks, uint64_t bs, uint32_t* d_bad,
                           hipStream_t s);
// Load each kernel file's code object onto the current device.  HIP loads a
// code object at the first launch of one of its kernels, ~10 ms on MI355X
// (tools/latency/first_call.py, profiles/r03z); xec_init does it instead, so
// the first codec call runs at the steady-state latency.
hipError_t preload_kernels();
hipError_t preload_validate();

}  // namespace xec
