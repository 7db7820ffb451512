// read_probe.hip -- how fast this HBM reads under different address geometries
// (a lab probe, NOT the product; standalone, no torch).
//
// Question: is the ~7.1 TB/s read-only rate measured on the encode's geometry
// (16 streams 1 MiB apart, tools/lab/lab.py --ceiling, profiles/r01w) the
// chip's read ceiling, or does the power-of-two member stride of the reference
// batch layout (abstract_bm.cpp:4-18: block i of stripe c at c*k*bs + i*bs)
// cost bandwidth that a different tile order could win back?
//
// Every kernel is the product's tile shape (csrc/xec_kernels.hip): one-wave
// workgroups, each lane one 16-B granule of a 1 KiB chunk, NM loads in flight
// per lane (all issued before the XOR), `nt` loads, the result stored only
// under a never-true test so the loads stay live.  Only the addresses differ:
//   tile t -> row r = t / tiles_per_row, chunk c = t % tiles_per_row,
//   load q at  r*row_stride + c*1024 + lane*16 + q*member_stride.
// Residency is capped as the product caps it (LDS reserved per workgroup).
//
// Build: make -C tools/lab read_probe   Run: tools/lab/read_probe [out.json]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Geo {
  uint64_t row_stride, member_stride, tiles_per_row, total_tiles;
  int reverse;  // walk tiles from the end (the product does)
  uint64_t alt_offset = 0;  // odd rows start this much further in (alternating classes)
  // row order: 0 as laid out; p > 0 interleaves p groups of rows/p rows
  // (consecutive tiles' rows are rows/p apart); -1 bit-reverses the row index
  int perm = 0;
  // column rotation: row r's chunk c reads column chunk
  // (c + r*rot) mod tiles_per_row, so the blocks of the rows in flight at
  // once are read at different offsets -- mixes the address bits of the
  // concurrently read blocks, where `perm` only changed which rows are in flight
  uint64_t rot = 0;
  // rows grouped: row r starts at (r / sub_rows) * row_stride + (r % sub_rows) *
  // sub_stride (encode with m > 1: the m classes of a stripe are rows 1 block
  // apart, stripes k blocks apart); 0 = rows row_stride apart
  uint64_t sub_rows = 0, sub_stride = 0;
  // XOR swizzle: row r's chunk c reads column
  // c ^ ((r * swz) mod tiles_per_row) (tiles_per_row a power of two)
  uint64_t swz = 0;
};

__device__ __forceinline__ uint64_t row_of(uint64_t r, const Geo& g) {
  const uint64_t rows = (g.total_tiles + g.tiles_per_row - 1) / g.tiles_per_row;
  if (g.perm > 0) return (r % g.perm) * (rows / g.perm) + r / g.perm;
  if (g.perm < 0) {
    uint64_t bits = 0;
    while ((1ull << bits) < rows) ++bits;
    return __brevll(r) >> (64 - bits);
  }
  return r;
}

template <int NM, bool NT>
__global__ __launch_bounds__(64) void read_kernel(const uint8_t* __restrict__ base, Geo g,
                                                  uint32_t magic, uint8_t* sink) {
  const uint64_t t0 = blockIdx.x;
  if (t0 >= g.total_tiles) return;
  const uint64_t t = g.reverse ? g.total_tiles - 1 - t0 : t0;
  const uint64_t r = row_of(t / g.tiles_per_row, g);
  uint64_t c = (t % g.tiles_per_row + r * g.rot) % g.tiles_per_row;
  if (g.swz) c ^= (r * g.swz) & (g.tiles_per_row - 1);
  const uint64_t row_base = g.sub_rows ? (r / g.sub_rows) * g.row_stride + (r % g.sub_rows) * g.sub_stride
                                       : r * g.row_stride + (r & 1) * g.alt_offset;
  const uint8_t* p = base + row_base + c * 1024 + threadIdx.x * 16;
  u32x4 v[NM];
#pragma unroll
  for (int q = 0; q < NM; ++q) {
    const u32x4* a = reinterpret_cast<const u32x4*>(p + (uint64_t)q * g.member_stride);
    v[q] = NT ? __builtin_nontemporal_load(a) : *a;
  }
  u32x4 acc = v[0];
#pragma unroll
  for (int q = 1; q < NM; ++q) acc ^= v[q];
  if (acc.x == magic && acc.y == magic && acc.z == magic && acc.w == magic)
    *reinterpret_cast<u32x4*>(sink + threadIdx.x * 16) = acc;
}

// write-only: each workgroup writes `per_wg` contiguous KiB (one 1 KiB
// wave-instruction per KiB), nt stores
__global__ __launch_bounds__(64) void write_kernel(uint8_t* base, uint64_t tiles, int per_wg,
                                                   uint32_t salt) {
  const uint64_t t = blockIdx.x;
  if (t >= tiles) return;
  uint8_t* p = base + t * (uint64_t)per_wg * 1024 + threadIdx.x * 16;
  for (int q = 0; q < per_wg; ++q) {
    const u32x4 v = {(uint32_t)t ^ salt, (uint32_t)q, threadIdx.x, salt};
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p + q * 1024));
  }
}

uint32_t lds_for_occupancy(int waves) {  // as csrc/xec_api.cpp, one-wave workgroups
  if (waves <= 0 || waves >= 8) return 0;
  uint32_t b = (160u * 1024u) / (uint32_t)(4 * waves);
  b &= ~511u;
  return b > 65536u ? 65536u : b;
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,          \
                   hipGetErrorString(e_));                                     \
      std::exit(2);                                                            \
    }                                                                          \
  } while (0)

struct Case {
  std::string name;
  int nm;
  bool nt;
  Geo g;
};

template <int NM, bool NT>
void launch_read(const Case& cs, const uint8_t* buf, uint8_t* sink, uint32_t lds, hipStream_t s) {
  read_kernel<NM, NT><<<dim3((uint32_t)cs.g.total_tiles), dim3(64), lds, s>>>(buf, cs.g, 0x9E3779B9u,
                                                                              sink);
}

void launch(const Case& cs, const uint8_t* buf, uint8_t* sink, uint32_t lds, hipStream_t s) {
  if (cs.nm == 16 && cs.nt) launch_read<16, true>(cs, buf, sink, lds, s);
  else if (cs.nm == 16) launch_read<16, false>(cs, buf, sink, lds, s);
  else if (cs.nm == 32 && cs.nt) launch_read<32, true>(cs, buf, sink, lds, s);
  else if (cs.nm == 8 && cs.nt) launch_read<8, true>(cs, buf, sink, lds, s);
  else if (cs.nm == 4 && cs.nt) launch_read<4, true>(cs, buf, sink, lds, s);
  else std::exit(3);
}

double median(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

}  // namespace

int main(int argc, char** argv) {
  const char* out = argc > 1 ? argv[1] : nullptr;
  const uint64_t KiB = 1024, MiB = KiB * KiB, GiB = MiB * KiB;
  std::vector<Case> cases;
  const uint64_t T16 = 4 * GiB / (16 * KiB);  // tiles of 16 x 1 KiB
  // the encode at config 3: 256 stripes x 16 blocks of 1 MiB
  cases.push_back({"cfg3_16x1MiB", 16, true, {16 * MiB, MiB, 1024, T16, 1}});
  cases.push_back({"cfg3_16x1MiB_fwd", 16, true, {16 * MiB, MiB, 1024, T16, 0}});
  cases.push_back({"cfg3_16x1MiB_default_policy", 16, false, {16 * MiB, MiB, 1024, T16, 1}});
  // the same, member stride not a power of two
  cases.push_back({"cfg3_members_1MiB+1KiB", 16, true, {16 * (MiB + KiB), MiB + KiB, 1024, T16, 1}});
  cases.push_back({"cfg3_members_1MiB+4KiB", 16, true, {16 * (MiB + 4 * KiB), MiB + 4 * KiB, 1024, T16, 1}});
  cases.push_back({"cfg3_members_1MiB+64KiB", 16, true, {16 * (MiB + 64 * KiB), MiB + 64 * KiB, 1024, T16, 1}});
  // stripes (rows) not a power of two apart, members 1 MiB
  cases.push_back({"cfg3_rows_16MiB+64KiB", 16, true, {16 * MiB + 64 * KiB, MiB, 1024, T16, 1}});
  // one wave reads 16 KiB contiguous (16 consecutive 1 KiB pieces)
  cases.push_back({"contig_16KiB_per_wave", 16, true, {16 * KiB, KiB, 1, T16, 1}});
  cases.push_back({"contig_16KiB_per_wave_default_policy", 16, false, {16 * KiB, KiB, 1, T16, 1}});
  // config 4's encode: 32 blocks of 4 KiB per stripe, 4 chunks per block
  cases.push_back({"cfg4_32x4KiB", 32, true, {128 * KiB, 4 * KiB, 4, 4 * GiB / (32 * KiB), 1}});
  // config 2's encode: 8 blocks of 64 KiB
  cases.push_back({"cfg2_8x64KiB", 8, true, {512 * KiB, 64 * KiB, 64, 4 * GiB / (8 * KiB), 1}});
  // the 16+2 x 1 MiB single-erasure decode's data reads: 8 blocks 2 MiB apart
  // in 16 MiB stripes, the class alternating from stripe to stripe (as the
  // bench's erasure pattern makes it), against the same class every stripe
  // and against 8 contiguous 1 MiB blocks
  const uint64_t T8 = 4 * GiB / (8 * KiB);
  cases.push_back({"d16p2_8x2MiB_alternating", 8, true, {16 * MiB, 2 * MiB, 1024, T8, 1, MiB}});
  cases.push_back({"d16p2_8x2MiB_same_class", 8, true, {16 * MiB, 2 * MiB, 1024, T8, 1, 0}});
  cases.push_back({"contig_8x1MiB", 8, true, {8 * MiB, MiB, 1024, T8, 1, 0}});
  // the same-class reads in other row orders (which stripes are in flight together)
  cases.push_back({"d16p2_same_class_rows_by2", 8, true, {16 * MiB, 2 * MiB, 1024, T8, 1, 0, 2}});
  cases.push_back({"d16p2_same_class_rows_by4", 8, true, {16 * MiB, 2 * MiB, 1024, T8, 1, 0, 4}});
  cases.push_back({"d16p2_same_class_rows_by16", 8, true, {16 * MiB, 2 * MiB, 1024, T8, 1, 0, 16}});
  cases.push_back({"d16p2_same_class_rows_bitrev", 8, true, {16 * MiB, 2 * MiB, 1024, T8, 1, 0, -1}});
  cases.push_back({"d16p2_alternating_rows_by4", 8, true, {16 * MiB, 2 * MiB, 1024, T8, 1, MiB, 4}});
  // column rotation of the same-class reads (one failed device: the same shard
  // lost in every stripe), R = rotation in 1 KiB chunks per stripe
  for (uint64_t R : {1ull, 3ull, 16ull, 64ull, 129ull, 256ull, 512ull})
    cases.push_back({"d16p2_same_class_rot" + std::to_string(R), 8, true,
                     {16 * MiB, 2 * MiB, 1024, T8, 1, 0, 0, R}});
  cases.push_back({"d16p2_alternating_rot64", 8, true, {16 * MiB, 2 * MiB, 1024, T8, 1, MiB, 0, 64}});
  // 8+2 x 1 MiB single erasure: 4 members 2 MiB apart in 8 MiB stripes
  const uint64_t T4 = 4 * GiB / (4 * KiB);
  cases.push_back({"d8p2_4x2MiB_same_class", 4, true, {8 * MiB, 2 * MiB, 1024, T4, 1, 0}});
  cases.push_back({"d8p2_4x2MiB_alternating", 4, true, {8 * MiB, 2 * MiB, 1024, T4, 1, MiB}});
  for (uint64_t R : {1ull, 64ull, 129ull, 512ull})
    cases.push_back({"d8p2_same_class_rot" + std::to_string(R), 4, true,
                     {8 * MiB, 2 * MiB, 1024, T4, 1, 0, 0, R}});
  // the encode's geometry rotated: must not lose (config 3)
  cases.push_back({"cfg3_16x1MiB_rot64", 16, true, {16 * MiB, MiB, 1024, T16, 1, 0, 0, 64}});
  // 32+4 x 1 MiB (the reference's (36/32) EC at the north star's shard size,
  // VERDICT r04 item 4): encode reads 8 members 4 MiB apart per class, the 4
  // classes of a stripe 1 MiB apart, stripes 32 MiB apart -- the same rows as
  // the random-loss decode's list tiles (one lost member of each class swapped
  // for its parity block; 7 of 8 loads keep this geometry)
  const uint64_t T8e = 4 * GiB / (8 * KiB);
  cases.push_back({"e32p4_8x4MiB", 8, true, {32 * MiB, 4 * MiB, 1024, T8e, 1, 0, 0, 0, 4, MiB}});
  cases.push_back({"e32p4_8x4MiB_fwd", 8, true, {32 * MiB, 4 * MiB, 1024, T8e, 0, 0, 0, 0, 4, MiB}});
  for (uint64_t R : {1ull, 3ull, 64ull, 257ull})
    cases.push_back({"e32p4_rowrot" + std::to_string(R), 8, true,
                     {32 * MiB, 4 * MiB, 1024, T8e, 1, 0, 0, R, 4, MiB}});
  for (uint64_t X : {1ull, 0x9E37ull, 0x2D5ull, 0x155ull})
    cases.push_back({"e32p4_swz" + std::to_string(X), 8, true,
                     {32 * MiB, 4 * MiB, 1024, T8e, 1, 0, 0, 0, 4, MiB, X}});
  // 16+2 x 1 MiB encode for comparison: 8 members 2 MiB apart, 2 classes 1 MiB apart
  cases.push_back({"e16p2_8x2MiB", 8, true, {16 * MiB, 2 * MiB, 1024, T8e, 1, 0, 0, 0, 2, MiB}});
  // the same 8 members as one contiguous 8 MiB run per class (no stride)
  cases.push_back({"e32p4_contig_8x1MiB", 8, true, {8 * MiB, MiB, 1024, T8e, 1, 0}});
  // cfg3's encode with the swizzle (the 16+1 shape must not lose)
  cases.push_back({"cfg3_16x1MiB_swz0x9E37", 16, true, {16 * MiB, MiB, 1024, T16, 1, 0, 0, 0, 0, 0, 0x9E37}});

  // Every byte a case reads must lie inside the buffers: the last tile's last
  // member ends at (rows-1)*row_stride + tiles_per_row*1 KiB + (nm-1)*member_stride.
  // The buffers are sized from that, checked again per case before it launches.
  uint64_t need = 0;
  auto end_of = [](const Case& cs) {
    const uint64_t rows = (cs.g.total_tiles + cs.g.tiles_per_row - 1) / cs.g.tiles_per_row;
    const uint64_t last_row =
        cs.g.sub_rows ? ((rows - 1) / cs.g.sub_rows) * cs.g.row_stride +
                            (cs.g.sub_rows - 1) * cs.g.sub_stride
                      : (rows - 1) * cs.g.row_stride + cs.g.alt_offset;
    return last_row + cs.g.tiles_per_row * 1024 + (uint64_t)(cs.nm - 1) * cs.g.member_stride;
  };
  for (const Case& cs : cases) need = std::max(need, end_of(cs));
  need = std::max(need, GiB);  // the write streams cover exactly 1 GiB
  need = (need + MiB - 1) / MiB * MiB;
  std::printf("buffers: 2 x %llu MiB\n", (unsigned long long)(need / MiB));
  uint8_t* bufs[2];
  for (auto& b : bufs) {
    CK(hipMalloc(&b, need));
    CK(hipMemset(b, 0x5A, need));
  }
  uint8_t* sink;
  CK(hipMalloc(&sink, 4096));
  hipStream_t s;
  CK(hipStreamCreate(&s));

  const int iters = 15;
  const int occs[] = {0, 2, 4};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::string json = "{\n \"note\": \"read-only rates by address geometry, tools/lab/read_probe.hip\",\n \"results\": [\n";
  bool first = true;
  auto emit = [&](const std::string& name, int occ, double bytes, double ms) {
    const double gbps = bytes / (ms * 1e-3) / 1e9;
    std::printf("%-40s occ %d  %8.4f ms  %7.1f GB/s\n", name.c_str(), occ, ms, gbps);
    std::fflush(stdout);
    char line[256];
    std::snprintf(line, sizeof line, "%s  {\"case\": \"%s\", \"waves_per_simd\": %d, \"ms_med\": %.4f, \"GBps_med\": %.1f}",
                  first ? "" : ",\n", name.c_str(), occ, ms, gbps);
    json += line;
    first = false;
  };
  const char* only = std::getenv("READ_PROBE_ONLY");  // substring filter on case names
  for (int round = 0; round < 2; ++round) {  // two interleaved passes
    for (const Case& cs : cases) {
      if (only && cs.name.find(only) == std::string::npos && cs.name.find("cfg3_16x1MiB") != 0)
        continue;
      if (end_of(cs) > need || cs.g.total_tiles > 0x7fffffffu) {
        std::fprintf(stderr, "case %s reaches %llu bytes of %llu: not launched\n", cs.name.c_str(),
                     (unsigned long long)end_of(cs), (unsigned long long)need);
        return 4;
      }
      for (int occ : occs) {
        const uint32_t lds = lds_for_occupancy(occ);
        launch(cs, bufs[0], sink, lds, s);  // warm-up
        std::vector<float> ts;
        for (int i = 0; i < iters; ++i) {
          CK(hipEventRecord(e0, s));
          launch(cs, bufs[(i + 1) % 2], sink, lds, s);
          CK(hipEventRecord(e1, s));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          ts.push_back(ms);
        }
        CK(hipGetLastError());
        emit(cs.name + (round ? "#2" : ""), occ,
             (double)cs.g.total_tiles * cs.nm * 1024.0, median(ts));
      }
    }
    // write-only streams of 1 GiB, 1 / 4 KiB contiguous per workgroup
    for (int per : {1, 4}) {
      if (only) break;
      for (int occ : occs) {
        const uint32_t lds = lds_for_occupancy(occ);
        const uint64_t tiles = GiB / ((uint64_t)per * KiB);  // tiles * per KiB = 1 GiB <= need
        std::vector<float> ts;
        for (int i = 0; i < iters + 1; ++i) {
          CK(hipEventRecord(e0, s));
          write_kernel<<<dim3((uint32_t)tiles), dim3(64), lds, s>>>(bufs[i % 2], tiles, per, i);
          CK(hipEventRecord(e1, s));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          if (i) ts.push_back(ms);
        }
        emit("write_1GiB_" + std::to_string(per) + "KiB_per_wg" + (round ? "#2" : ""), occ,
             (double)GiB, median(ts));
      }
    }
  }
  json += "\n ]\n}\n";
  if (out) {
    FILE* f = std::fopen(out, "w");
    if (f) {
      std::fputs(json.c_str(), f);
      std::fclose(f);
    }
  }
  for (auto b : bufs) CK(hipFree(b));
  CK(hipFree(sink));
  return 0;
}
