// xec_kernels.h -- internal interface between the C ABI (xec_api.cpp) and the
// gfx950 kernels (xec_kernels.hip).  Not part of the public boundary.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace xec {

constexpr int kThreads = 256;  // 4 waves of 64 lanes per workgroup

// Batch geometry, all in 16-byte granules except where named *_bytes.
struct Geometry {
  uint64_t S;                // stripes
  uint64_t k, m, nm;         // data blocks, parity blocks, members per class (k/m)
  uint64_t gran;             // granules per block (bs / 16)
  uint64_t tiles_per_block;  // ceil(gran / (kThreads * unroll))
  uint64_t total_tiles;      // S * m * tiles_per_block
};

struct LaunchShape {
  int unroll;         // granules per thread per member: 1, 2 or 4
  uint32_t max_grid;  // 0 = one workgroup per tile
  bool nt;            // non-temporal loads/stores
};

inline Geometry make_geometry(uint64_t S, uint64_t bs, uint64_t k, uint64_t m, int unroll) {
  Geometry g;
  g.S = S;
  g.k = k;
  g.m = m;
  g.nm = k / m;
  g.gran = bs / 16;
  uint64_t tile = (uint64_t)kThreads * (uint64_t)unroll;
  g.tiles_per_block = (g.gran + tile - 1) / tile;
  g.total_tiles = S * m * g.tiles_per_block;
  return g;
}

inline uint32_t grid_for(uint64_t work_items, uint32_t max_grid) {
  uint64_t cap = max_grid ? (uint64_t)max_grid : (uint64_t)0x7fffffffu;
  uint64_t grid = work_items < cap ? work_items : cap;
  return (uint32_t)(grid ? grid : 1);
}

hipError_t launch_encode(const void* d_data, void* d_parity, const Geometry& g,
                         const LaunchShape& ls, hipStream_t s);
hipError_t launch_decode(void* d_data, const void* d_parity, const uint8_t* d_bitmap,
                         const Geometry& g, const LaunchShape& ls, hipStream_t s);
hipError_t launch_erase(void* d_data, void* d_parity, const uint8_t* d_bitmap, const Geometry& g,
                        hipStream_t s);
hipError_t launch_fill(void* d_buf, uint64_t S, uint64_t words, uint64_t seed_base,
                       hipStream_t s);

}  // namespace xec
