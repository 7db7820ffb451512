// xec_api.cpp -- the C ABI of libxec_hip.so (declared in include/xec.h).
//
// Host-side responsibilities, each following the reference behaviour:
//   - initialisation contract        xorec_gpu_cmp.cu:7-27, xorec.cpp:16-22
//   - argument checks                xorec_utils.hpp:61-86
//   - batch recoverability scan      xorec_gpu_cmp.cu:75-81 (require_recovery /
//                                    is_recoverable, xorec_utils.hpp:144-175)
//   - H2D bitmap / work-list upload  xorec_gpu_cmp.cu:83 (here off the caller's
//                                    stream, upload_begin below)
// then one kernel launch per call (xec_kernels.hip).
#include "xec.h"

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "xec_internal.h"
#include "xec_kernels.h"

namespace {

std::atomic<bool> g_initialised{false};

// Tuning overrides (xec_set_launch, xec_set_occupancy, xec_set_decode_tiling);
// 0 = default.  Per thread: an override applies to the calls its own thread
// makes, so a tuning sweep on one thread never changes the kernels that
// another thread (a ShardPool worker, a pipeline user) launches meanwhile.
thread_local int g_unroll = 0;
thread_local int g_max_grid = 0;
thread_local int g_nt = 0;
thread_local int g_threads = 0;
thread_local int g_occupancy = 0;      // waves per SIMD, 0 = automatic
thread_local int g_decode_tiling = 0;  // 0 auto, 1 stripe, 2 class, 3 list, 4 mask
thread_local int g_arg_cap_used = 0;   // xec_decode_arg_capacity_used
thread_local int g_tiling_used = 0;    // xec_decode_tiling_used: this thread's last xec_decode
thread_local int g_rotation = 0;       // xec_set_rotation: 0 automatic, -1 none, > 0 tiles

constexpr size_t kBlockMultiple = 256;  // XOREC_BLOCK_SIZE_MULTIPLE
constexpr size_t kMinBlock = 256;       // XOREC_MIN_BLOCK_SIZE
constexpr size_t kAlign = 64;           // XOREC_ALIGNMENT
constexpr int kMaxRotation = 1 << 20;   // xec_set_rotation's upper bound (tiles)

// LDS to reserve per workgroup so that at most `waves` waves of T-thread
// workgroups are resident per SIMD: a gfx950 CU has 160 KiB of LDS and 4
// SIMDs, so 4*waves/(T/64) workgroups fit.  Rounded down to the 512-B
// allocation granule (7 waves per SIMD comes out as 7.25); 0 = no cap.
uint32_t lds_for_occupancy(int waves, int threads) {
  if (waves <= 0 || waves >= 8) return 0;
  const uint32_t wgs = (uint32_t)(4 * waves) / (uint32_t)(threads / 64);
  uint32_t b = wgs ? (160u * 1024u) / wgs : 65536u;
  b &= ~511u;
  return b > 65536u ? 65536u : b;
}

// Resident waves per SIMD that measured fastest for the default shape (one
// wave per workgroup, one granule per lane), by class member count k/m
// (bf0ca45:tools/archive/sweep.py --occ; profiles/r01i, r01j: two devices, encode and decode,
// k=4..32).  A wave keeps up to k/m KiB of loads in flight (~11 KiB at k/m =
// 16, hipcc's rolling window; all 32 at k/m = 32); the best residency keeps
// roughly 16-32 KiB in flight per SIMD -- 8 waves per SIMD at k/m = 16 queue
// 4x the requests and ran 3 % (encode) to 6 % (decode) slower.  0 = no cap
// (8 per SIMD).  Member counts without a compiled unroll run the generic loop
// (8 loads in flight per group); swept at 3, 5, 6, 12, 24, 48 and 64
// (profiles/r02q): no cap below 8 members, 4 waves from 8 (12: +6 / +5 %
// encode / decode), 2 from 20 (24: +8 / +8 %, 48: +4 / +7 %), 1 from 56
// (64: +6 / +3 %).
int auto_occupancy(uint64_t nm) {
  switch (nm) {
    case 1: case 2: return 0;
    case 4: case 8: return 4;
    case 16: return 2;
    case 32: return 1;
    default: return nm < 8 ? 0 : nm < 20 ? 4 : nm < 56 ? 2 : 1;
  }
}

// Decode does one class reduction per lost data block of its stripe, one after
// the other, so its work per tile is k/m x (lost blocks per stripe) loads.  At
// one erasure per stripe that is the encode table above; with several
// (bf0ca45:tools/archive/sweep.py --lost, profiles/r01p: 16+2, 16+4, 16+8, 32+8, 8+2 at 2..8
// erasures per stripe) 2 waves per SIMD measured best from 8 loads per tile
// up (+3 to +15 % over the single-erasure choice), 4 from 4.  Only the member
// counts those shapes cover (2, 4, 8) take this branch.
// The policy reads the batch average, i.e. it assumes the losses are spread
// evenly over the stripes (as in every measured shape); a batch where a few
// stripes lose many blocks and most lose none is classed as single-erasure.
int decode_auto_occupancy(uint64_t nm, uint64_t lost_data, uint64_t S) {
  if (lost_data <= S || (nm != 2 && nm != 4 && nm != 8)) return auto_occupancy(nm);
  const uint64_t work = nm * ((lost_data + S - 1) / S);
  return work >= 8 ? 2 : work >= 4 ? 4 : 0;
}

// Decode tiling (xec_kernels.hip).  List tiles (the default where the list
// fits, below) give every lost data block its own tiles: one reduction each,
// none idle, whatever the spread of the losses.  Otherwise, stripe tiles run
// one class reduction per lost data block of their stripe, back to back;
// class tiles are encode's tiles, one reduction each, but a class without a
// loss leaves its tiles idle.  Measured in one process on both (bf0ca45:tools/archive/tiling_ab.py,
// profiles/r02a/tiling_ab.json; 16+2, 8+2 x 1 MiB, 16+4, 16+8, 32+8 x 64 KiB at
// 1, m/2 and m losses per stripe): class tiles win once more than one block
// per stripe AND at least half of the classes are lost (+3 to +9 % with every
// class lost, +16 % at 16+8 with 4 lost, tie at 32+8 with 4), and lose
// clearly below that (-6 % at 8+2 with one loss per stripe, 3x slower at
// 16+8 with one).  With m == 1 the tilings coincide.
bool use_class_tiles(uint64_t S, uint64_t m, uint64_t lost_data) {
  const int t = g_decode_tiling;
  if (m <= 1 || t == 1) return false;
  if (t == 2) return true;
  return lost_data > S && 2 * lost_data >= S * m;  // automatic (0, or 3 / 4 where n/a)
}

// ---- work-list staging -------------------------------------------------------
// The work list is written by the host scan into pinned host memory and copied
// into the caller's d_bitmap scratch on the stream.  A staging buffer is
// reused once the copy queued from it has run (its event); buffers are kept
// for the life of the process (a copy may still be queued when a call
// returns), at most kMaxStaging per process unless every one is in use.
struct Staging {
  void* host = nullptr;
  size_t cap = 0;
  int device = -1;
  hipEvent_t done = nullptr;     // on a library stream: the buffer's last reader has passed
  hipEvent_t handoff = nullptr;  // throw-away record on the caller's stream (record_after)
  bool busy = false;
};
constexpr size_t kMaxStaging = 64;
std::mutex g_stage_mu;
std::vector<Staging*> g_stage;

// The thread's pending HIP error and the library.  What
// the runtime does (tools/lab/last_error_probe.hip, profiles/r05b): a call
// that succeeds leaves a pending error alone; a call that fails replaces it;
// hipErrorNotReady from a stream or event query is not recorded on ROCm 7.2,
// but was read back as a launch failure under an earlier runtime
// (profiles/r04s).  So the library (1) asks no query at all while an error of
// the caller's is pending -- it takes the answer that needs none, which is
// always correct -- (2) clears a NotReady only if that is what the query left
// pending, and (3) reports any other query error as the call's failure,
// leaving it pending for the caller.
bool caller_error_pending() { return hipPeekAtLastError() != hipSuccess; }

void clear_own_not_ready() {
  if (hipPeekAtLastError() == hipErrorNotReady) (void)hipGetLastError();
}

// hipEventQuery on a buffer's event (recorded on a stream the library owns,
// track_stream below): 1 once the work it marks has passed, 0 not yet, -1 the
// query failed -- a sticky device fault, which fails the call.  The query is
// asked even while an error of the caller's is pending: taking
// every buffer as in use then made each call allocate a new one up to the
// pool's cap and then wait on a recycled one.  On this runtime a successful
// query leaves the pending error alone and a NotReady is not recorded
// (profiles/r05b), so only the clearing step is skipped: the pending error is
// the caller's, never ours to clear.
int event_passed(hipEvent_t e) {
  const bool callers = caller_error_pending();
  const hipError_t q = hipEventQuery(e);
  if (q == hipSuccess) return 1;
  if (q == hipErrorNotReady) {
    if (!callers) clear_own_not_ready();
    return 0;
  }
  return -1;
}

// A buffer read by the caller's stream is free once that stream has passed
// the reading work -- but an event recorded on the CALLER's stream may outlive
// that stream (a pipeline destroys its streams), and querying it later made
// HIP report a stray error (hipErrorStreamCaptureUnsupported, read by the
// next launch's hipGetLastError: tools/fuzz_big.py --pipeline, profiles/r04s).
// So the caller's stream only hands over to a tracking stream of the
// library's (hipStreamWaitEvent on a throw-away record), and the buffer's
// event is recorded there.  A tracking stream waits for its callers in the
// order the hand-offs were queued, so one shared stream would keep a short
// decode's buffer busy behind every earlier caller's unrelated long work
// (ADVICE r04): each device has kTrackLanes of them, a caller stream always
// hands over to the same lane (its handle hashed), so independent callers on
// different streams rarely share one (g_track_mu guards the list).
constexpr size_t kTrackLanes = 4;
std::mutex g_track_mu;
struct TrackLanes {
  int dev;
  hipStream_t lane[kTrackLanes];
};
std::vector<TrackLanes> g_track_streams;
hipStream_t track_stream(int dev, hipStream_t caller) {
  const uintptr_t h = reinterpret_cast<uintptr_t>(caller);
  const size_t lane = static_cast<size_t>((h >> 4) ^ (h >> 12)) % kTrackLanes;
  std::lock_guard<std::mutex> lk(g_track_mu);
  for (auto& ts : g_track_streams)
    if (ts.dev == dev) return ts.lane[lane];
  TrackLanes t{dev, {}};
  for (auto& s : t.lane)
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
      for (auto& made : t.lane)
        if (made != nullptr) (void)hipStreamDestroy(made);
      return nullptr;
    }
  g_track_streams.push_back(t);
  return t.lane[lane];
}

// Record `done` once `caller` has passed its current work, on a tracking
// stream of `dev` (`handoff` is the throw-away record on the caller's
// stream); false if that cannot be queued.
bool record_after(hipEvent_t done, hipEvent_t handoff, hipStream_t caller, int dev) {
  const hipStream_t ts = track_stream(dev, caller);
  return ts != nullptr && hipEventRecord(handoff, caller) == hipSuccess &&
         hipStreamWaitEvent(ts, handoff, 0) == hipSuccess && hipEventRecord(done, ts) == hipSuccess;
}

// The slot is picked and marked busy under the lock; waiting for a recycled
// buffer's last reader and re-allocating happen after the lock is dropped, so
// one thread waiting for another's copy never stalls other threads' calls.
// *fault: an event query failed (event_passed -1); nullptr is returned and
// the call must fail.
Staging* stage_acquire(size_t bytes, int dev, bool* fault) {
  Staging* pick = nullptr;
  bool recycled = false;
  {
    std::lock_guard<std::mutex> lk(g_stage_mu);
    for (Staging* st : g_stage) {
      if (st->busy || st->device != dev || st->cap < bytes) continue;
      const int passed = event_passed(st->done);
      if (passed < 0) {
        *fault = true;
        return nullptr;
      }
      if (passed == 0) continue;  // a queued copy still reads it
      if (pick == nullptr || st->cap < pick->cap) pick = st;
    }
    if (pick == nullptr && g_stage.size() >= kMaxStaging) {
      for (Staging* st : g_stage)  // recycle an idle one of this device: wait for its copy
        if (!st->busy && st->device == dev) {
          pick = st;
          recycled = true;
          break;
        }
    }
    if (pick == nullptr) {
      pick = new Staging;
      pick->device = dev;
      if (hipEventCreateWithFlags(&pick->done, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&pick->handoff, hipEventDisableTiming) != hipSuccess) {
        if (pick->done) (void)hipEventDestroy(pick->done);
        delete pick;
        return nullptr;
      }
      g_stage.push_back(pick);
    }
    pick->busy = true;
  }
  auto give_back = [&]() {
    std::lock_guard<std::mutex> lk(g_stage_mu);
    pick->busy = false;
    return nullptr;
  };
  if (recycled && hipEventSynchronize(pick->done) != hipSuccess) {
    *fault = true;  // a sticky fault: left pending for the caller
    return give_back();
  }
  if (pick->cap < bytes) {
    if (pick->host != nullptr) (void)hipHostFree(pick->host);
    pick->host = nullptr;
    pick->cap = 0;
    size_t cap = 64u << 10;
    while (cap < bytes) cap <<= 1;
    if (hipHostMalloc(&pick->host, cap, hipHostMallocDefault) != hipSuccess) {
      pick->host = nullptr;
      return give_back();
    }
    pick->cap = cap;
  }
  return pick;
}

// `stream` = where a copy from the buffer was queued (nullptr-able), or
// `queued` = false when nothing was; `own`: the stream is the library's (its
// copy stream), else the caller's (record_after).  If the event cannot be
// recorded, the copy is waited for instead, so the buffer is never reused early.
void stage_release(Staging* st, bool queued, hipStream_t stream, bool own) {
  if (queued && !(own ? hipEventRecord(st->done, stream) == hipSuccess
                      : record_after(st->done, st->handoff, stream, st->device)))
    (void)hipStreamSynchronize(stream);
  std::lock_guard<std::mutex> lk(g_stage_mu);
  st->busy = false;
}

// ---- uploads off the caller's stream ---------------------------------------
// What a decode kernel reads besides the batch -- the bitmap or the work list
// -- comes from host memory.  Copied on the caller's stream, the copy waits
// for the kernel before it and the decode kernel for the copy (the copy
// engine's start and completion hand-offs included): 17-73 us per decode in
// tools/lab/mix_ceiling.py (profiles/r03f: event time minus kernel time at
// 16+8, 32+8, 32+1 x 4 KiB), 2-8 % of those decodes.  So the bytes go to a
// device buffer the library owns, on a copy stream of its own (one per
// device, non-blocking), which starts at once -- while the caller's stream is
// still busy with earlier work -- and the decode kernel only waits for the
// copy's event.  A buffer is reused once the kernel that read it has passed
// (its event on the caller's stream); buffers are kept for the life of the
// process, at most kMaxSlots per device unless every one is in use.  The
// caller's d_bitmap scratch is used instead when no buffer can be had.
struct DevSlot {
  void* dev = nullptr;
  size_t cap = 0;
  int device = -1;
  hipEvent_t copied = nullptr;  // on the copy stream, after the upload
  hipEvent_t done = nullptr;    // on a library stream, after the reading kernel (record_after)
  hipEvent_t handoff = nullptr;  // throw-away record on the caller's stream
  bool busy = false;
};
constexpr size_t kMaxSlots = 16;
std::mutex g_slot_mu;
std::vector<DevSlot*> g_slots;
std::vector<std::pair<int, hipStream_t>> g_copy_streams;

hipStream_t copy_stream(int dev) {  // under g_slot_mu
  for (auto& cs : g_copy_streams)
    if (cs.first == dev) return cs.second;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  g_copy_streams.emplace_back(dev, s);
  return s;
}

struct Upload {
  DevSlot* slot = nullptr;  // null: the bytes went to the caller's scratch on `stream`
  hipStream_t cs = nullptr;  // the copy stream they went on
  uint8_t* dev = nullptr;   // where the kernel reads them
};

// XEC_SCRATCH_UPLOADS=1 in the environment sends every upload through the
// caller's scratch on the stream (the fallback path; tests use it).
bool side_uploads() {
  static const bool off = [] {
    const char* e = std::getenv("XEC_SCRATCH_UPLOADS");
    return e != nullptr && e[0] == '1';
  }();
  return !off;
}

// Uploads go off the caller's stream only while that stream is busy: then a
// copy queued on it would wait for the kernel before it (the bubble above).
// On an idle stream -- a synchronous caller such as the reference's
// BM_generic loop, which synchronises after every call -- the copy on the
// stream starts at once, and the side path's cross-stream event would only
// add latency: 8 MiB (40/32) with 8 lost ran at 2,284 instead of 3,669
// Gbit/s per call, 128 MiB with 2-8 lost 21-27 % slower (tools/ab/
// refrows_ab.sh, profiles/r03zk).  A NotReady answer is cleared so that no
// later hipGetLastError reads it as a launch failure; any other answer (a
// sticky fault of earlier work, an invalid stream) is an error the caller
// gets back as XEC_DEVICE_ERROR, and is left for its hipGetLastError.  While
// an error of the caller's is pending nothing is asked: the stream is taken as
// idle (the copy goes on it, correct either way) and the error stays theirs.
// Returns 0 idle, 1 busy, -1 error.
int stream_busy(hipStream_t stream) {
  if (caller_error_pending()) return 0;
  const hipError_t q = hipStreamQuery(stream);
  if (q == hipSuccess) return 0;
  if (q != hipErrorNotReady) {
    if (const char* e = std::getenv("XEC_DEBUG"); e != nullptr && e[0] == '1')
      std::fprintf(stderr, "xec: hipStreamQuery: %s\n", hipGetErrorName(q));
    return -1;
  }
  clear_own_not_ready();
  return 1;
}

// The device `stream` belongs to (the current device for the null stream).
// HIP accepts a stream of device B while device A is current, and the decode
// kernel then runs on B: the library buffers, copy stream and staging the
// call uses must be B's too.  So a decode makes the stream's device current
// for its duration and restores the caller's on return.
class StreamDevice {
 public:
  explicit StreamDevice(hipStream_t stream) {
    ok_ = hipGetDevice(&prev_) == hipSuccess;
    dev_ = prev_;
    if (ok_ && stream != nullptr) {
      ok_ = hipStreamGetDevice(stream, &dev_) == hipSuccess;
      if (ok_ && dev_ != prev_) ok_ = switched_ = hipSetDevice(dev_) == hipSuccess;
    }
  }
  ~StreamDevice() {
    if (switched_) (void)hipSetDevice(prev_);
  }
  StreamDevice(const StreamDevice&) = delete;
  StreamDevice& operator=(const StreamDevice&) = delete;
  bool ok() const { return ok_; }
  int device() const { return dev_; }

 private:
  int prev_ = 0, dev_ = 0;
  bool ok_ = false, switched_ = false;
};

bool capturing(hipStream_t stream) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(stream, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone;
}

// Starts copying `bytes` of host memory to a library buffer on the device's
// copy stream; false (nothing queued) if no buffer or stream can be had, and
// then *fault if an event query or wait failed (the call must fail).
// `dev` is the current device (StreamDevice).  As in stage_acquire, a slot is
// picked and marked busy under the lock, and a recycled slot's wait and
// re-allocation happen outside it.
bool upload_begin(const void* host, size_t bytes, int dev, Upload& up, bool* fault) {
  DevSlot* pick = nullptr;
  hipStream_t cs = nullptr;
  bool recycled = false;
  {
    std::lock_guard<std::mutex> lk(g_slot_mu);
    cs = copy_stream(dev);
    if (cs == nullptr) return false;
    for (DevSlot* sl : g_slots) {
      if (sl->busy || sl->device != dev || sl->cap < bytes) continue;
      const int passed = event_passed(sl->done);
      if (passed < 0) {
        *fault = true;
        return false;
      }
      if (passed == 0) continue;  // a kernel still reads it
      if (pick == nullptr || sl->cap < pick->cap) pick = sl;
    }
    size_t mine = 0;
    for (DevSlot* sl : g_slots) mine += sl->device == dev;
    if (pick == nullptr && mine >= kMaxSlots) {
      for (DevSlot* sl : g_slots)  // recycle an idle one: wait for its reader (below)
        if (!sl->busy && sl->device == dev) {
          pick = sl;
          recycled = true;
          break;
        }
      if (pick == nullptr) return false;
    }
    if (pick == nullptr) {
      pick = new DevSlot;
      pick->device = dev;
      if (hipEventCreateWithFlags(&pick->copied, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&pick->done, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&pick->handoff, hipEventDisableTiming) != hipSuccess) {
        if (pick->copied) (void)hipEventDestroy(pick->copied);
        if (pick->done) (void)hipEventDestroy(pick->done);
        delete pick;
        return false;
      }
      g_slots.push_back(pick);
    }
    pick->busy = true;
  }
  auto give_back = [&]() {
    std::lock_guard<std::mutex> lk(g_slot_mu);
    pick->busy = false;
    return false;
  };
  if (recycled && hipEventSynchronize(pick->done) != hipSuccess) {
    *fault = true;  // a sticky fault: left pending for the caller
    return give_back();
  }
  if (pick->cap < bytes) {
    if (pick->dev != nullptr) (void)hipFree(pick->dev);
    pick->dev = nullptr;
    pick->cap = 0;
    size_t cap = 64u << 10;
    while (cap < bytes) cap <<= 1;
    if (hipMalloc(&pick->dev, cap) != hipSuccess) {
      pick->dev = nullptr;
      return give_back();
    }
    pick->cap = cap;
  }
  if (hipMemcpyAsync(pick->dev, host, bytes, hipMemcpyHostToDevice, cs) != hipSuccess ||
      hipEventRecord(pick->copied, cs) != hipSuccess) {
    (void)hipStreamSynchronize(cs);
    std::lock_guard<std::mutex> lk(g_slot_mu);
    pick->busy = false;
    return false;
  }
  up.slot = pick;
  up.cs = cs;
  up.dev = static_cast<uint8_t*>(pick->dev);
  return true;
}

// The caller's stream waits for the upload (before the kernel that reads it).
bool upload_join(const Upload& up, hipStream_t stream) {
  return up.slot == nullptr || hipStreamWaitEvent(stream, up.slot->copied, 0) == hipSuccess;
}

// After the launch (`launched`: a kernel on `stream` reads the buffer) or
// without one: the buffer is free once that kernel, or the copy, has passed.
void upload_end(Upload& up, hipStream_t stream, bool launched) {
  if (up.slot == nullptr) return;
  hipStream_t after = launched ? stream : up.cs;
  const bool ok = launched ? record_after(up.slot->done, up.slot->handoff, stream, up.slot->device)
                           : hipEventRecord(up.slot->done, up.cs) == hipSuccess;
  if (!ok) (void)hipStreamSynchronize(after);
  std::lock_guard<std::mutex> lk(g_slot_mu);
  up.slot->busy = false;
  up.slot = nullptr;
}

// Defaults measured on MI355X (bf0ca45:tools/archive/sweep.py, profiles/r01_sweep_*.json):
// non-temporal loads and parity stores, sc1 rebuilt-block stores (every byte
// is touched once; xec_kernels.hip kEncodeStoreAux / kDecodeStoreAux), one-wave
// workgroups with one 1 KiB tile each, one workgroup per tile, residency
// capped per member count (auto_occupancy).
// Column rotation of the tile kernels (Geometry::rot): the chunks a stripe's
// column walk is shifted by, per stripe (xec_set_rotation).  Automatic: none
// for encode and for decodes the host scan cannot see; decode_rotation below.
uint32_t rotation() {
  const int r = g_rotation;
  return r > 0 ? (uint32_t)r : 0u;
}

// Automatic decode rotation.  When every lost data block of the batch sits in
// one parity class -- one failed device: the same shard gone from every
// stripe -- with m >= 2, the stripes in flight read the same columns of k/m
// blocks m*bs apart, which this HBM serves slowly; an odd rotation puts them
// on different columns.  Measured in one process against no rotation
// (tools/lab/loss_pattern_probe.py --rotations, profiles/r04d): one failed
// device +15.7 % at 16+2 x 1 MiB, +15.4 % at 8+2, +11.5 % at 16+4, +5.8 % at
// 32+4, +5.4 % at 16+2 x 512 KiB, +3.8 % at 16+2 x 4 MiB, but -4.0 % at
// 16+2 x 256 KiB -- hence the 512 KiB floor.  Where the class alternates
// between stripes (the bench's pattern) or several classes lost blocks, a
// rotation lost up to 11 %, and encode lost 2-15 % (profiles/r04c), so neither
// rotates.
// The lost_class of a work list (xec_decode_per_stripe lists the rebuilt
// blocks only; its scan has no class summary of its own).
XecScan items_scan(const uint32_t* items, uint64_t n, size_t m) {
  XecScan v;
  v.lost_data = n;
  for (uint64_t q = 0; q < n; ++q) {
    const int64_t c = static_cast<int64_t>((items[q] & 0xFFu) % m);
    if (q == 0) v.lost_class = c;
    else if (v.lost_class != c) {
      v.lost_class = -1;
      break;
    }
  }
  return v;
}

constexpr uint32_t kSameClassRotation = 3;
constexpr size_t kRotateMinBlock = 512u << 10;
uint32_t decode_rotation(const XecScan& scan, size_t m, size_t bs) {
  const int r = g_rotation;
  if (r != 0) return r > 0 ? (uint32_t)r : 0u;
  return m >= 2 && scan.lost_class >= 0 && bs >= kRotateMinBlock ? kSameClassRotation : 0u;
}

xec::LaunchShape launch_shape(size_t bs, int auto_w) {
  xec::LaunchShape ls;
  ls.rot = rotation();
  const int t = g_threads;
  ls.threads = t == 256 ? 256 : 64;
  const int u = g_unroll;
  ls.unroll = (u == 1 || u == 2) ? u : 1;
  const int g = g_max_grid;
  ls.max_grid = g > 0 ? (uint32_t)g : 0u;
  // nt stores address the block with a 32-bit buffer offset (xec_kernels.hip)
  ls.nt = g_nt != 2 && bs <= 0x7fffffffu;
  int w = g_occupancy;
  if (w == 0) w = (ls.threads == 64 && ls.unroll == 1) ? auto_w : 0;
  ls.lds_bytes = lds_for_occupancy(w, ls.threads);
  return ls;
}

// Workgroups the chip holds at once for a launch of shape ls (CUs x the
// workgroups per CU its LDS reservation admits, at most 32 waves per CU):
// the fixed grid of decode_devlist_kernel, which walks a count the host never
// sees.  0 if the device cannot be queried.
constexpr uint64_t kDevListMaxGrid = 131072;  // xec_decode_device_list's largest default grid

uint32_t resident_workgroups(const xec::LaunchShape& ls) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    return 0;
  const uint32_t waves = (uint32_t)ls.threads / 64u;
  uint32_t per_cu = 32u / (waves ? waves : 1u);
  if (ls.lds_bytes > 0 && (160u * 1024u) / ls.lds_bytes < per_cu)
    per_cu = (160u * 1024u) / ls.lds_bytes;
  return (uint32_t)cus * (per_cu ? per_cu : 1u);
}

}  // namespace

extern "C" {

xec_status xec_check_args(const void* data, const void* parity, size_t bs, size_t k, size_t m) {
  if (reinterpret_cast<uintptr_t>(data) % kAlign != 0 ||
      reinterpret_cast<uintptr_t>(parity) % kAlign != 0)
    return XEC_INVALID_ALIGNMENT;
  if (bs < kMinBlock || bs % kBlockMultiple != 0) return XEC_INVALID_SIZE;
  if (k < 1 || m < 1 || k % m != 0) return XEC_INVALID_COUNTS;
  return XEC_SUCCESS;
}

// xec_check_bitmap / xec_scan_bitmap live in xec_scan.cpp (host-only, AVX2 where available).

xec_status xec_init(int device_id) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return XEC_DEVICE_ERROR;
  if (device_id < 0 || device_id >= count) return XEC_DEVICE_ERROR;
  if (hipSetDevice(device_id) != hipSuccess) return XEC_DEVICE_ERROR;
  // code objects onto the device now rather than at the first codec call
  if (xec::preload_kernels() != hipSuccess || xec::preload_validate() != hipSuccess)
    return XEC_DEVICE_ERROR;
  g_initialised.store(true, std::memory_order_release);
  return XEC_SUCCESS;
}

// xec_set_kernel_events arms the next codec call of this thread; that call
// consumes the setting whether or not it launched a kernel (include/xec.h).
struct KernelEventsScope {
  ~KernelEventsScope() { xec::t_kernel_events = xec::KernelEvents{}; }
};

xec_status xec_set_kernel_events(hipEvent_t start, hipEvent_t stop) {
  xec::t_kernel_events = xec::KernelEvents{start, stop};
  return XEC_SUCCESS;
}

xec_status xec_encode(const void* d_data, void* d_parity, size_t S, size_t bs, size_t k, size_t m,
                      hipStream_t stream) {
  const KernelEventsScope events_scope;
  if (!g_initialised.load(std::memory_order_acquire)) return XEC_NOT_INITIALIZED;
  xec_status st = xec_check_args(d_data, d_parity, bs, k, m);
  if (st != XEC_SUCCESS) return st;
  if (S == 0) return XEC_SUCCESS;
  const xec::LaunchShape ls = launch_shape(bs, auto_occupancy(k / m));
  const xec::Geometry g = xec::make_geometry(S, bs, k, m, ls);
  return xec::launch_encode(d_data, d_parity, g, ls, stream) == hipSuccess ? XEC_SUCCESS
                                                                           : XEC_DEVICE_ERROR;
}

// Bitmaps from this size on are copied to the device BEFORE the host scan, so
// the scan (~1.1 ns per stripe, 75 us for config 4's 65,536 stripes) runs
// while the transfer does and the synchronous caller waits for
// max(scan, copy) + kernel instead of their sum (bf0ca45:tools/archive/scan_cost.py,
// profiles/r02b, r02c).  Smaller bitmaps keep the scan first, so a batch that
// needs no recovery queues no device work at all.
constexpr size_t kCopyFirstBitmapBytes = 256u << 10;

// Work-list tiles are taken (automatic tiling) when at most this fraction of
// the stripes lost a data block: then stripe and class tiles would leave most
// of their tiles idle (sparse: 2.2x faster at 1 stripe in 9, skewed: 1.0-3.1x
// at 1 in 5; bf0ca45:tools/archive/tiling_ab.py --pattern, profiles/r02n).  When every stripe
// lost blocks, the bitmap tilings are as fast or faster (list tiles -1..-5 %
// against the better of them, profiles/r02n/tiling_uniform.json, r02o).
constexpr uint64_t kListStripesNum = 3, kListStripesDen = 4;

// XEC_DEBUG=1: a decode that fails with XEC_DEVICE_ERROR names its line, the
// HIP error of the failing call and the one pending on the thread (stderr;
// diagnostics only).
static bool debug_on() {
  static const bool on = [] {
    const char* e = std::getenv("XEC_DEBUG");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}
static xec_status dev_error(int line, hipError_t e) {
  if (debug_on())
    std::fprintf(stderr, "xec: device error at xec_api.cpp:%d (%s; pending %s)\n", line,
                 hipGetErrorName(e), hipGetErrorName(hipPeekAtLastError()));
  return XEC_DEVICE_ERROR;
}
#define DEVERR(e) dev_error(__LINE__, (e))

static xec_status decode_impl(void* d_data, const void* d_parity, size_t S, size_t bs, size_t k,
                              size_t m, const uint8_t* h_bitmap, uint8_t* d_bitmap,
                              hipStream_t stream) {
  g_tiling_used = 0;
  g_arg_cap_used = 0;
  if (!g_initialised.load(std::memory_order_acquire)) return XEC_NOT_INITIALIZED;
  xec_status st = xec_check_args(d_data, d_parity, bs, k, m);
  if (st != XEC_SUCCESS) return st;
  if (S == 0) return XEC_SUCCESS;
  const size_t bitmap_bytes = S * (k + m);
  // The host scan reads h_bitmap now: a graph captured from this call would
  // replay this call's losses whatever the bitmap holds then.  So a call with
  // work to queue is refused on a capturing stream, before anything is
  // queued; xec_decode_device is the capturable form.  A batch that needs no
  // recovery, or cannot be recovered, returns its verdict from the scan
  // alone, before any device call -- the reference's order
  // (xorec_gpu_cmp.cu:75-81) -- so it never pays the capture query.
  const bool cap = bitmap_bytes >= kCopyFirstBitmapBytes && capturing(stream);
  const bool copy_first = bitmap_bytes >= kCopyFirstBitmapBytes && !cap;
  // Small bitmaps are scanned first: a batch that needs no recovery (or
  // cannot be recovered) returns before any device query or copy.  That pass
  // also lists the lost data blocks, speculatively, so a decode whose list
  // travels in the kernel arguments -- the small messages, e.g. the
  // reference's 8 MiB rows -- scans its bitmap once, not twice (VERDICT r05
  // item 3: the second pass was ~0.6-0.8 us of an 8 MiB decode call).  The
  // scan stops listing once its projection says the list will not be used
  // (more than kArgItems losses, or a class-tile batch): listing 1,024 items
  // for nothing cost 1.3 us (profiles/r06i).
  XecScan scan;
  uint32_t items[xec::kArgItems];
  bool listed = false;  // items holds every lost data block
  if (!copy_first) {
    st = xec_scan_bitmap(h_bitmap, S, k, m, &scan, items, xec::kArgItems, /*speculative=*/true);
    listed = scan.listed == scan.lost_data;
    if (st != XEC_SUCCESS || !scan.needs_recovery || scan.lost_data == 0) return st;
    if (cap || capturing(stream)) return DEVERR(hipSuccess);
  }
  const StreamDevice sd(stream);
  if (!sd.ok()) return DEVERR(hipSuccess);
  const int dev = sd.device();
  // Whether uploads go off the stream, asked (hipStreamQuery) only when
  // something is about to be uploaded: a list that travels in the kernel
  // arguments never pays for the query.  A query that fails (not merely
  // "busy") fails the call.
  int side_state = -2;
  bool query_failed = false;
  auto side = [&]() {
    if (side_state == -2) {
      side_state = side_uploads() ? stream_busy(stream) : 0;
      query_failed = side_state < 0;
    }
    return side_state == 1;
  };
  // The bitmap goes to the device (a library buffer, or the caller's scratch
  // on `stream`); for large bitmaps before the scan, so the two overlap.
  Upload bmu;
  auto upload_bitmap = [&]() -> bool {
    if (side() && upload_begin(h_bitmap, bitmap_bytes, dev, bmu, &query_failed)) return true;
    if (query_failed) return false;
    bmu = Upload{};
    bmu.dev = d_bitmap;
    return hipMemcpyAsync(d_bitmap, h_bitmap, bitmap_bytes, hipMemcpyHostToDevice, stream) ==
           hipSuccess;
  };
  if (copy_first) {
    if (!upload_bitmap()) return DEVERR(hipSuccess);
    st = xec_scan_bitmap(h_bitmap, S, k, m, &scan, nullptr, 0);
    if (st != XEC_SUCCESS || !scan.needs_recovery || scan.lost_data == 0) {
      upload_end(bmu, stream, false);  // only the bitmap copy was queued
      return st;                       // failure, or nothing to rebuild
    }
  }
  // Which tiling: list tiles when the losses are sparse (or forced); for a
  // list short enough to travel in the kernel arguments also wherever stripe
  // tiles would run (no copy at all); class tiles keep dense multi-erasure
  // batches.  The list is built by a second, listing pass only
  // when it is used (the first pass costs ~1.1 ns per stripe).
  const int tiling = g_decode_tiling;
  const bool listable = (tiling == 0 || tiling == 3 || tiling == 4) && k <= kWorkItemMaxK &&
                        S <= kWorkItemMaxStripes;
  const bool small = scan.lost_data <= xec::kArgItems;
  const bool sparse = scan.stripes_lost * kListStripesDen <= (uint64_t)S * kListStripesNum;
  const bool cls = use_class_tiles(S, m, scan.lost_data);
  // A batch of at most kArgItems stripes (k <= 32) whose decode would upload
  // something -- a list longer than the kernel arguments hold, or the bitmap
  // for class / stripe tiles -- sends one loss mask per stripe in the kernel
  // arguments instead, over class tiles where the bitmap path would take them
  // and stripe tiles otherwise: nothing is copied, so a synchronous caller
  // does not wait for a copy ahead of the kernel (decode_argmask_kernel; the
  // reference's row 1126, 8 MiB (40/32) with 8 losses, profiles/r06w).  Forced
  // with xec_set_decode_tiling(4).
  const bool arglist = listable && small && (tiling == 3 || sparse || !cls);
  const bool maskable = !copy_first && S <= xec::kArgItems && k <= xec::kArgMaskMaxK;
  if (maskable && (tiling == 4 || (tiling == 0 && !arglist))) {
    uint32_t masks[xec::kArgItems];
    xec_loss_masks(h_bitmap, S, k, m, masks);
    // class tiles: one reduction per tile, encode's residency table; stripe
    // tiles: as the bitmap's stripe tiles
    xec::LaunchShape ls = launch_shape(
        bs, cls ? auto_occupancy(k / m) : decode_auto_occupancy(k / m, scan.lost_data, S));
    ls.rot = decode_rotation(scan, m, bs);
    const xec::Geometry g = xec::make_geometry(S, bs, k, m, ls);
    g_tiling_used = cls ? XEC_TILING_ARG_MASK : XEC_TILING_ARG_MASK_STRIPE;
    g_arg_cap_used = (int)xec::arg_items_capacity(S);
    const hipError_t le = xec::launch_decode(
        d_data, d_parity, nullptr, g, ls,
        cls ? xec::kDecodeArgMaskTiles : xec::kDecodeArgMaskStripeTiles, stream, S, masks);
    return le == hipSuccess ? XEC_SUCCESS : DEVERR(le);
  }
  if (listable && (tiling == 3 || sparse || (!cls && small))) {
    // one reduction per tile, as encode: encode's residency table
    xec::LaunchShape ls = launch_shape(bs, auto_occupancy(k / m));
    ls.rot = decode_rotation(scan, m, bs);
    const xec::Geometry g = xec::make_geometry(S, bs, k, m, ls);
    if (small) {  // the launch copies the list into its kernel arguments
      upload_end(bmu, stream, false);
      if (!listed) {
        st = xec_scan_bitmap(h_bitmap, S, k, m, &scan, items, xec::kArgItems);
        if (st != XEC_SUCCESS) return st;
      }
      g_tiling_used = XEC_TILING_ARG_LIST;
      g_arg_cap_used = (int)xec::arg_items_capacity(scan.lost_data);
      const hipError_t le = xec::launch_decode(d_data, d_parity, nullptr, g, ls,
                                               xec::kDecodeArgListTiles, stream, scan.lost_data,
                                               items);
      return le == hipSuccess ? XEC_SUCCESS : DEVERR(le);
    }
    // u32 entries staged in pinned host memory by the listing pass, then
    // uploaded: to a library buffer off the stream, or into the 4-byte-aligned
    // part of the caller's S*(k+m)-byte scratch on it (if the list fits)
    const size_t pad = (4 - reinterpret_cast<uintptr_t>(d_bitmap) % 4) % 4;
    const uint64_t cap = bitmap_bytes > pad ? (bitmap_bytes - pad) / 4 : 0;
    const uint64_t n = scan.lost_data;
    Staging* sg = nullptr;
    const bool off_stream = side();
    if (query_failed) {
      upload_end(bmu, stream, false);
      return DEVERR(hipSuccess);
    }
    if (off_stream || n <= cap) sg = stage_acquire(n * 4, dev, &query_failed);
    if (query_failed) {
      upload_end(bmu, stream, false);
      return DEVERR(hipSuccess);
    }
    if (sg != nullptr) {
      st = xec_scan_bitmap(h_bitmap, S, k, m, &scan, static_cast<uint32_t*>(sg->host), n);
      if (st != XEC_SUCCESS) {
        stage_release(sg, false, stream, false);
        upload_end(bmu, stream, false);
        return st;
      }
      Upload lu;
      bool ok = true;
      if (side() && upload_begin(sg->host, n * 4, dev, lu, &query_failed)) {
        stage_release(sg, true, lu.cs, true);
        ok = upload_join(lu, stream);
      } else if (query_failed) {
        stage_release(sg, false, stream, false);
        upload_end(bmu, stream, false);
        return DEVERR(hipSuccess);
      } else if (n <= cap) {
        // stream-ordered after any bitmap copy into the same scratch
        lu.dev = d_bitmap + pad;
        ok = hipMemcpyAsync(lu.dev, sg->host, n * 4, hipMemcpyHostToDevice, stream) == hipSuccess;
        stage_release(sg, ok, stream, false);
      } else {
        stage_release(sg, false, stream, false);  // denser than the scratch holds: bitmap tiles
      }
      if (lu.dev != nullptr) {
        upload_end(bmu, stream, false);
        g_tiling_used = XEC_TILING_LIST;
        const hipError_t le =
            ok ? xec::launch_decode(d_data, d_parity, lu.dev, g, ls, xec::kDecodeListTiles,
                                    stream, n)
               : hipErrorUnknown;
        upload_end(lu, stream, true);
        return le == hipSuccess ? XEC_SUCCESS : DEVERR(le);
      }
    }
    // no staging memory, or a list denser than the scratch holds: bitmap tiles
  }
  if (!copy_first && !upload_bitmap()) return DEVERR(hipSuccess);
  if (!upload_join(bmu, stream)) {
    upload_end(bmu, stream, false);
    return DEVERR(hipSuccess);
  }
  // class tiles: one reduction per tile, so the encode's residency table
  xec::LaunchShape ls = launch_shape(
      bs, cls ? auto_occupancy(k / m) : decode_auto_occupancy(k / m, scan.lost_data, S));
  ls.rot = decode_rotation(scan, m, bs);
  const xec::Geometry g = xec::make_geometry(S, bs, k, m, ls);
  g_tiling_used = cls && m > 1 ? XEC_TILING_CLASS : XEC_TILING_STRIPE;
  const hipError_t le = xec::launch_decode(d_data, d_parity, bmu.dev, g, ls,
                                           cls ? xec::kDecodeClassTiles : xec::kDecodeStripeTiles,
                                           stream);
  upload_end(bmu, stream, true);
  return le == hipSuccess ? XEC_SUCCESS : DEVERR(le);
}

// No exception crosses the C ABI: the host-side bookkeeping allocates (upload
// buffers, pinned staging, their lists), and an allocation failure there is a
// device error for the caller, not a std::terminate.
xec_status xec_decode(void* d_data, const void* d_parity, size_t S, size_t bs, size_t k, size_t m,
                      const uint8_t* h_bitmap, uint8_t* d_bitmap, hipStream_t stream) {
  const KernelEventsScope events_scope;
  try {
    return decode_impl(d_data, d_parity, S, bs, k, m, h_bitmap, d_bitmap, stream);
  } catch (...) {
    return XEC_DEVICE_ERROR;
  }
}

int xec_decode_tiling_used(void) { return g_tiling_used; }
int xec_decode_arg_capacity_used(void) { return g_arg_cap_used; }

static xec_status decode_per_stripe_impl(void* d_data, const void* d_parity, size_t S, size_t bs,
                                         size_t k, size_t m, const uint8_t* h_bitmap,
                                         uint8_t* d_bitmap, uint8_t* h_codes, hipStream_t stream) {
  g_tiling_used = 0;
  g_arg_cap_used = 0;
  if (!g_initialised.load(std::memory_order_acquire)) return XEC_NOT_INITIALIZED;
  xec_status st = xec_check_args(d_data, d_parity, bs, k, m);
  if (st != XEC_SUCCESS) return st;
  if (S == 0) return XEC_SUCCESS;
  if (k > kWorkItemMaxK || S > kWorkItemMaxStripes) return XEC_INVALID_SIZE;
  uint64_t n = 0, failures = 0;
  // one pass gives the verdicts and, for a short list, the list itself
  uint32_t short_items[xec::kArgItems];
  st = xec_scan_stripes(h_bitmap, S, k, m, h_codes, short_items, xec::kArgItems, &n, &failures);
  if (st != XEC_SUCCESS) return st;
  const xec_status verdict = failures ? XEC_DECODE_FAILURE : XEC_SUCCESS;
  if (n == 0) return verdict;
  if (capturing(stream)) return XEC_DEVICE_ERROR;  // work to queue: see xec_decode
  xec::LaunchShape ls = launch_shape(bs, auto_occupancy(k / m));
  xec::Geometry g = xec::make_geometry(S, bs, k, m, ls);
  // the rebuilt blocks' classes decide the column rotation, as in xec_decode
  auto rotate_for = [&](const uint32_t* items, uint64_t count) {
    ls.rot = decode_rotation(items_scan(items, count, m), m, bs);
    g = xec::make_geometry(S, bs, k, m, ls);
  };
  if (n <= xec::kArgItems) {
    rotate_for(short_items, n);
    g_tiling_used = XEC_TILING_ARG_LIST;
    g_arg_cap_used = (int)xec::arg_items_capacity(n);
    return xec::launch_decode(d_data, d_parity, nullptr, g, ls, xec::kDecodeArgListTiles, stream,
                              n, short_items) == hipSuccess
               ? verdict
               : XEC_DEVICE_ERROR;
  }
  // A longer list is uploaded whole off the stream (upload_begin), or else
  // goes through the scratch in pieces of what it holds: copy a piece, rebuild
  // it, copy the next (stream order keeps a copy behind the kernel still
  // reading the previous piece).
  const StreamDevice sd(stream);  // the stream's device, as in xec_decode
  if (!sd.ok()) return XEC_DEVICE_ERROR;
  const int dev = sd.device();
  const int busy = side_uploads() ? stream_busy(stream) : 0;
  if (busy < 0) return XEC_DEVICE_ERROR;
  bool fault = false;
  Staging* sg = stage_acquire(n * 4, dev, &fault);
  if (sg == nullptr) return XEC_DEVICE_ERROR;
  uint32_t* items = static_cast<uint32_t*>(sg->host);
  (void)xec_scan_stripes(h_bitmap, S, k, m, nullptr, items, n, &n, &failures);
  rotate_for(items, n);
  g_tiling_used = XEC_TILING_LIST;
  Upload lu;
  if (busy == 1 && upload_begin(items, n * 4, dev, lu, &fault)) {
    stage_release(sg, true, lu.cs, true);
    const bool ok = upload_join(lu, stream) &&
                    xec::launch_decode(d_data, d_parity, lu.dev, g, ls, xec::kDecodeListTiles,
                                       stream, n) == hipSuccess;
    upload_end(lu, stream, true);
    return ok ? verdict : XEC_DEVICE_ERROR;
  }
  if (fault) {  // an event query or wait failed in upload_begin
    stage_release(sg, false, stream, false);
    return XEC_DEVICE_ERROR;
  }
  const size_t pad = (4 - reinterpret_cast<uintptr_t>(d_bitmap) % 4) % 4;
  const uint64_t cap = (S * (k + m) - pad) / 4;  // >= 511 here: n > 1,024 <= S*k
  uint8_t* d_items = d_bitmap + pad;
  bool queued = false, ok = true;
  for (uint64_t q0 = 0; q0 < n && ok; q0 += cap) {
    const uint64_t piece = n - q0 < cap ? n - q0 : cap;
    ok = hipMemcpyAsync(d_items, items + q0, piece * 4, hipMemcpyHostToDevice, stream) ==
         hipSuccess;
    queued |= ok;
    ok = ok && xec::launch_decode(d_data, d_parity, d_items, g, ls, xec::kDecodeListTiles, stream,
                                  piece) == hipSuccess;
  }
  stage_release(sg, queued, stream, false);
  return ok ? verdict : XEC_DEVICE_ERROR;
}

xec_status xec_decode_per_stripe(void* d_data, const void* d_parity, size_t S, size_t bs,
                                 size_t k, size_t m, const uint8_t* h_bitmap, uint8_t* d_bitmap,
                                 uint8_t* h_codes, hipStream_t stream) {
  const KernelEventsScope events_scope;
  try {  // as xec_decode
    return decode_per_stripe_impl(d_data, d_parity, S, bs, k, m, h_bitmap, d_bitmap, h_codes,
                                  stream);
  } catch (...) {
    return XEC_DEVICE_ERROR;
  }
}

xec_status xec_decode_device(void* d_data, const void* d_parity, size_t S, size_t bs, size_t k,
                             size_t m, const uint8_t* d_bitmap, int32_t* d_status,
                             hipStream_t stream) {
  const KernelEventsScope events_scope;
  if (!g_initialised.load(std::memory_order_acquire)) return XEC_NOT_INITIALIZED;
  xec_status st = xec_check_args(d_data, d_parity, bs, k, m);
  if (st != XEC_SUCCESS) return st;
  // every argument is checked before any work is queued on the stream
  if (d_status == nullptr || reinterpret_cast<uintptr_t>(d_status) % 4 != 0)
    return XEC_INVALID_ALIGNMENT;
  if (d_bitmap == nullptr && S != 0) return XEC_INVALID_SIZE;
  if (hipMemsetAsync(d_status, 0, sizeof(int32_t), stream) != hipSuccess) return XEC_DEVICE_ERROR;
  if (S == 0) return XEC_SUCCESS;
  // No host view of the bitmap: the loss count is unknown, so the tiling is
  // the stripe tiling with the single-erasure residency table unless
  // xec_set_decode_tiling(2) says every class lost a block.
  const bool cls = m > 1 && g_decode_tiling == 2;
  const xec::LaunchShape ls = launch_shape(bs, auto_occupancy(k / m));
  xec::Geometry g = xec::make_geometry(S, bs, k, m, ls);
  if (xec::launch_check(d_bitmap, g, d_status, stream) != hipSuccess) return XEC_DEVICE_ERROR;
  g.gate = d_status;
  return xec::launch_decode(d_data, d_parity, d_bitmap, g, ls,
                            cls ? xec::kDecodeClassTiles : xec::kDecodeStripeTiles,
                            stream) == hipSuccess
             ? XEC_SUCCESS
             : XEC_DEVICE_ERROR;
}

size_t xec_decode_device_list_bytes(size_t S, size_t k, size_t m) {
  (void)k;
  return 4 * (xec::kDevListHeader + S * m);
}

xec_status xec_decode_device_list(void* d_data, const void* d_parity, size_t S, size_t bs,
                                  size_t k, size_t m, const uint8_t* d_bitmap, void* d_work,
                                  size_t work_bytes, int32_t* d_status, hipStream_t stream) {
  const KernelEventsScope events_scope;
  if (!g_initialised.load(std::memory_order_acquire)) return XEC_NOT_INITIALIZED;
  xec_status st = xec_check_args(d_data, d_parity, bs, k, m);
  if (st != XEC_SUCCESS) return st;
  // every argument is checked before any work is queued on the stream
  if (d_status == nullptr || reinterpret_cast<uintptr_t>(d_status) % 4 != 0 ||
      d_work == nullptr || reinterpret_cast<uintptr_t>(d_work) % 4 != 0)
    return XEC_INVALID_ALIGNMENT;
  if (S != 0 && (d_bitmap == nullptr || k > kWorkItemMaxK || S > kWorkItemMaxStripes ||
                 work_bytes < xec_decode_device_list_bytes(S, k, m)))
    return XEC_INVALID_SIZE;
  if (S == 0)
    return hipMemsetAsync(d_status, 0, sizeof(int32_t), stream) == hipSuccess ? XEC_SUCCESS
                                                                              : XEC_DEVICE_ERROR;
  // One reduction per tile, as encode: encode's residency table.  The list's
  // length is known only on the device, so the decode walks it with a grid
  // fixed at launch (unless xec_set_launch gave max_grid): one workgroup per
  // 8 possible tiles (S*m entries x chunks), at least what the chip holds at
  // once (on the stream's device) and at most kDevListMaxGrid.  A grid past
  // the list's end costs ~0.17 ns per idle workgroup; a grid of only what the
  // chip holds walks a dense list 5-18 % slower than one workgroup per tile.
  // Against that resident-only grid this was 3-5 % faster on dense lists and
  // 1-8 % on sparse ones (configs 2-4, 16+8 x 64 KiB, every stripe or 1 in 9
  // losing a block; tools/lab/devlist_grid.py, profiles/r06n).
  const StreamDevice sd(stream);
  if (!sd.ok()) return XEC_DEVICE_ERROR;
  xec::LaunchShape ls = launch_shape(bs, auto_occupancy(k / m));
  xec::Geometry g = xec::make_geometry(S, bs, k, m, ls);
  if (ls.max_grid == 0) {
    const uint64_t resident = resident_workgroups(ls);
    if (resident == 0) return XEC_DEVICE_ERROR;
    const uint64_t eighth = (uint64_t)S * m * g.tiles_per_block / 8;
    const uint64_t want = eighth < kDevListMaxGrid ? eighth : kDevListMaxGrid;
    ls.max_grid = (uint32_t)(want > resident ? want : resident);
  }
  uint32_t* list = static_cast<uint32_t*>(d_work);
  if (xec::launch_scan_list(d_bitmap, g, d_status, list, stream) != hipSuccess)
    return XEC_DEVICE_ERROR;
  g.gate = d_status;
  return xec::launch_decode(d_data, d_parity, reinterpret_cast<const uint8_t*>(list), g, ls,
                            xec::kDecodeDevListTiles, stream, S * m) == hipSuccess
             ? XEC_SUCCESS
             : XEC_DEVICE_ERROR;
}

xec_status xec_erase(void* d_data, void* d_parity, size_t S, size_t bs, size_t k, size_t m,
                     const uint8_t* d_bitmap, hipStream_t stream) {
  if (!g_initialised.load(std::memory_order_acquire)) return XEC_NOT_INITIALIZED;
  xec_status st = xec_check_args(d_data, d_parity, bs, k, m);
  if (st != XEC_SUCCESS) return st;
  if (S == 0) return XEC_SUCCESS;
  const xec::Geometry g = xec::make_geometry(S, bs, k, m, xec::LaunchShape{256, 1, 0, false, 0});
  return xec::launch_erase(d_data, d_parity, d_bitmap, g, stream) == hipSuccess ? XEC_SUCCESS
                                                                               : XEC_DEVICE_ERROR;
}

xec_status xec_fill_splitmix64(void* d_buf, size_t S, size_t stripe_bytes, uint64_t seed_base,
                               hipStream_t stream) {
  if (!g_initialised.load(std::memory_order_acquire)) return XEC_NOT_INITIALIZED;
  if (reinterpret_cast<uintptr_t>(d_buf) % 8 != 0) return XEC_INVALID_ALIGNMENT;
  if (stripe_bytes % 8 != 0) return XEC_INVALID_SIZE;
  return xec::launch_fill(d_buf, S, stripe_bytes / 8, seed_base, stream) == hipSuccess
             ? XEC_SUCCESS
             : XEC_DEVICE_ERROR;
}

xec_status xec_write_validation_pattern(void* d_data, size_t nblocks, size_t bs, uint64_t seed,
                                        hipStream_t stream) {
  if (!g_initialised.load(std::memory_order_acquire)) return XEC_NOT_INITIALIZED;
  if (bs < 2) return XEC_INVALID_SIZE;
  if (bs >= 16 && bs % 16 == 0 && reinterpret_cast<uintptr_t>(d_data) % 16 != 0)
    return XEC_INVALID_ALIGNMENT;
  return xec::launch_pattern(d_data, nblocks, bs, seed, stream) == hipSuccess ? XEC_SUCCESS
                                                                              : XEC_DEVICE_ERROR;
}

xec_status xec_validate_blocks(const void* d_data, size_t nblocks, size_t bs, uint32_t* d_bad,
                               hipStream_t stream) {
  if (!g_initialised.load(std::memory_order_acquire)) return XEC_NOT_INITIALIZED;
  if (bs >= 16 && bs % 16 == 0 && reinterpret_cast<uintptr_t>(d_data) % 16 != 0)
    return XEC_INVALID_ALIGNMENT;
  if (reinterpret_cast<uintptr_t>(d_bad) % 4 != 0) return XEC_INVALID_ALIGNMENT;
  return xec::launch_validate(d_data, nblocks, bs, d_bad, stream) == hipSuccess
             ? XEC_SUCCESS
             : XEC_DEVICE_ERROR;
}

xec_status xec_set_launch(int unroll, int max_grid, int cache_policy, int block_threads) {
  if (unroll != 0 && unroll != 1 && unroll != 2) return XEC_INVALID_SIZE;
  if (max_grid < 0 || cache_policy < 0 || cache_policy > 2) return XEC_INVALID_SIZE;
  if (block_threads != 0 && block_threads != 64 && block_threads != 256) return XEC_INVALID_SIZE;
  g_threads = block_threads;
  g_unroll = unroll;
  g_max_grid = max_grid;
  g_nt = cache_policy;
  return XEC_SUCCESS;
}

xec_status xec_set_occupancy(int waves_per_simd) {
  if (waves_per_simd < 0 || waves_per_simd > 8) return XEC_INVALID_SIZE;
  g_occupancy = waves_per_simd;
  return XEC_SUCCESS;
}

xec_status xec_set_decode_tiling(int tiling) {
  if (tiling < 0 || tiling > 4) return XEC_INVALID_SIZE;
  g_decode_tiling = tiling;
  return XEC_SUCCESS;
}

xec_status xec_set_validate_kernel(int mode) {
  if (mode < 0 || mode > 2) return XEC_INVALID_SIZE;
  xec::g_validate_mode = mode;
  return XEC_SUCCESS;
}

xec_status xec_set_rotation(int tiles) {
  if (tiles < -1 || tiles > kMaxRotation) return XEC_INVALID_SIZE;
  g_rotation = tiles;
  return XEC_SUCCESS;
}

xec_status xec_get_tuning(xec_tuning* out) {
  if (out == nullptr) return XEC_INVALID_ALIGNMENT;
  out->rotation = g_rotation;
  out->unroll = g_unroll;
  out->max_grid = g_max_grid;
  out->cache_policy = g_nt;
  out->block_threads = g_threads;
  out->waves_per_simd = g_occupancy;
  out->decode_tiling = g_decode_tiling;
  out->validate_kernel = xec::g_validate_mode;
  return XEC_SUCCESS;
}

xec_status xec_set_tuning(const xec_tuning* in) {
  if (in == nullptr) return XEC_INVALID_ALIGNMENT;
  // all or nothing: each setter checks its own fields; if any rejects, the
  // thread's previous values are put back
  const xec_tuning keep = [] {
    xec_tuning t{};
    (void)xec_get_tuning(&t);
    return t;
  }();
  if (xec_set_launch(in->unroll, in->max_grid, in->cache_policy, in->block_threads) !=
          XEC_SUCCESS ||
      xec_set_occupancy(in->waves_per_simd) != XEC_SUCCESS ||
      xec_set_decode_tiling(in->decode_tiling) != XEC_SUCCESS ||
      xec_set_validate_kernel(in->validate_kernel) != XEC_SUCCESS ||
      xec_set_rotation(in->rotation) != XEC_SUCCESS) {
    g_unroll = keep.unroll;
    g_max_grid = keep.max_grid;
    g_nt = keep.cache_policy;
    g_threads = keep.block_threads;
    g_occupancy = keep.waves_per_simd;
    g_decode_tiling = keep.decode_tiling;
    xec::g_validate_mode = keep.validate_kernel;
    g_rotation = keep.rotation;
    return XEC_INVALID_SIZE;
  }
  return XEC_SUCCESS;
}

const char* xec_status_string(xec_status s) {
  switch (s) {
    case XEC_SUCCESS: return "Success";
    case XEC_INVALID_SIZE: return "InvalidSize";
    case XEC_INVALID_ALIGNMENT: return "InvalidAlignment";
    case XEC_INVALID_COUNTS: return "InvalidCounts";
    case XEC_DECODE_FAILURE: return "DecodeFailure";
    case XEC_NOT_INITIALIZED: return "NotInitialized";
    case XEC_DEVICE_ERROR: return "DeviceError";
  }
  return "Unknown";
}

#ifndef XEC_SRC_ID
#define XEC_SRC_ID "unknown"
#endif
// "src:<id>": the hash of the library's sources (erasure-code-benchmark_amd/Makefile)
xec_status xec_peer_link(int device, int peer, xec_peer_link_info* out) {
  int n = 0;
  if (out == nullptr) return XEC_INVALID_COUNTS;
  if (hipGetDeviceCount(&n) != hipSuccess) return XEC_DEVICE_ERROR;
  if (device < 0 || peer < 0 || device >= n || peer >= n) return XEC_INVALID_COUNTS;
  xec_peer_link_info r{1, -1, -1};
  if (device != peer) {
    if (hipDeviceCanAccessPeer(&r.can_access_peer, device, peer) != hipSuccess)
      return XEC_DEVICE_ERROR;
    uint32_t type = 0, hops = 0;
    // A pair the runtime knows no link for reports an error: that is "none",
    // not a failure of this call.  The error is ours to clear -- unless one
    // of the caller's was pending, which stays where it was (DESIGN.md §7,
    // the thread's error state).
    const bool clean = hipPeekAtLastError() == hipSuccess;
    if (hipExtGetLinkTypeAndHopCount(device, peer, &type, &hops) == hipSuccess) {
      r.link_type = (int)type;
      r.hop_count = (int)hops;
    } else if (clean) {
      (void)hipGetLastError();
    }
  }
  *out = r;
  return XEC_SUCCESS;
}

const char* xec_build_info(void) { return "xec-hip gfx950 src:" XEC_SRC_ID " " __DATE__ " " __TIME__; }

}  // extern "C"
