// xec_pipeline.cpp -- host-in / host-out XOR-EC.
//
// The MI355X analogue of the reference's GPU-memory / unified-memory
// variants (src/algorithms/xorec_gpu_ptr_bm.cpp:17-65,
// xorec_unified_ptr_bm.cpp:15-86), which move data between host and device
// and compute on the CPU.  Here the data starts and ends in (pinned) host
// memory and the codec runs on the GPU: the batch is cut into chunks of
// `chunk_stripes` stripes and each chunk goes
//     H2D (data [+ parity])  ->  kernel  ->  D2H (parity | recovered blocks)
// on one of `nstreams` streams with its own device slot, so chunk i's copies
// overlap chunk i±1's copies and kernels.  PCIe, not HBM, bounds this path.
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "xec.h"
#include "xec_kernels.h"

namespace {

// Results bound for PAGEABLE host memory (file or socket buffers).  A D2H
// copy into pageable memory is staged by HIP and holds the calling thread
// until the stream reaches it and the bytes are out: ~75 us per 1 MiB rebuilt
// block at config 3, in series with the next chunk's (also host-synchronous)
// input copies (rocprofv3 trace, profiles/r03v).  So such results go to a
// pinned bounce buffer per slot (an asynchronous DMA) and this helper thread
// moves them to their destinations once the copy's event has passed, while
// the caller's thread already copies the next chunk in.
class HostCopier {
 public:
  struct Piece {
    uint8_t* dst;
    const uint8_t* src;
    size_t bytes;
  };
  HostCopier(int device, size_t nslots) : device_(device), busy_(nslots, 0) {
    th_ = std::thread([this] { run(); });
  }
  ~HostCopier() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();  // the queue is drained first
  }
  // After `ev` has passed, copy `pieces` (out of slot's bounce buffer).
  void push(size_t slot, hipEvent_t ev, std::vector<Piece>&& pieces) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      ++busy_[slot];
      q_.push_back(Job{slot, ev, std::move(pieces)});
    }
    cv_.notify_all();
  }
  // The slot's bounce buffer (and its event) may be reused.
  void wait_slot(size_t slot) {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return busy_[slot] == 0; });
  }
  // Every queued copy done; false if an event wait failed since the last drain.
  bool drain() {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] {
      for (size_t b : busy_)
        if (b) return false;
      return true;
    });
    const bool ok = !failed_;
    failed_ = false;
    return ok;
  }

 private:
  struct Job {
    size_t slot;
    hipEvent_t ev;
    std::vector<Piece> pieces;
  };
  void run() {
    (void)hipSetDevice(device_);
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        j = std::move(q_.front());
        q_.pop_front();
      }
      const bool ok = hipEventSynchronize(j.ev) == hipSuccess;
      if (ok)
        for (const Piece& pc : j.pieces) std::memcpy(pc.dst, pc.src, pc.bytes);
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (!ok) failed_ = true;
        --busy_[j.slot];
      }
      done_cv_.notify_all();
    }
  }
  int device_;
  std::vector<size_t> busy_;  // queued jobs per slot
  std::deque<Job> q_;
  bool stop_ = false, failed_ = false;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::thread th_;
};

// Inputs from PAGEABLE host memory.  A H2D copy from pageable memory is
// staged by HIP and holds the calling thread until its bytes are out, so the
// copy engine idles whenever this thread does anything else (the next
// chunk's scan and launch, the previous chunk's copy-out): pageable decode
// 48.8 against pinned 55.1 GB/s at config 3, with each of the two inputs
// costing its share (profiles/r03u, r03w).  So the inputs of the NEXT chunk
// are copied into a pinned staging buffer by this pool of host threads while
// the current chunk's DMA runs, and every H2D copy reads pinned memory.
// Jobs are numbered by staging buffer; a buffer holds one job at a time.
class HostPool {
 public:
  using Piece = HostCopier::Piece;
  // A thread that cannot be started leaves none behind: the ones already
  // running are stopped and joined before the exception leaves the
  // constructor (no destructor runs then, and a joinable std::thread would
  // terminate the process instead of reaching ensure_stage's catch).
  HostPool(int device, unsigned threads, size_t jobs)
      : device_(device), left_(jobs, 0), failed_(jobs, 0) {
    try {
      for (unsigned t = 0; t < threads; ++t) th_.emplace_back([this] { run(); });
    } catch (...) {
      stop_all();
      throw;
    }
  }
  ~HostPool() { stop_all(); }
  // Once `after` has passed (null: at once), copy `pieces`, cut into tasks of
  // at most kTaskBytes so that every thread takes a share.  Job `j` must be
  // idle (wait(j) returned since its last submit).
  void submit(size_t j, hipEvent_t after, const std::vector<Piece>& pieces) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      failed_[j] = 0;
      for (const Piece& pc : pieces)
        for (size_t o = 0; o < pc.bytes; o += kTaskBytes) {
          const size_t b = pc.bytes - o < kTaskBytes ? pc.bytes - o : kTaskBytes;
          q_.push_back(Task{j, after, Piece{pc.dst + o, pc.src + o, b}});
          ++left_[j];
        }
    }
    cv_.notify_all();
  }
  // Job j done; false if its event could not be waited for.
  bool wait(size_t j) {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return left_[j] == 0; });
    return failed_[j] == 0;
  }
  void drain() {
    for (size_t j = 0; j < left_.size(); ++j) (void)wait(j);
  }

 private:
  static constexpr size_t kTaskBytes = 2u << 20;
  void stop_all() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();  // the queue is drained first
    th_.clear();
  }
  struct Task {
    size_t job;
    hipEvent_t after;
    Piece pc;
  };
  void run() {
    (void)hipSetDevice(device_);
    for (;;) {
      Task t;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        t = q_.front();
        q_.pop_front();
      }
      // the staging buffer's previous DMA has read it (returns at once once passed)
      const bool ok = t.after == nullptr || hipEventSynchronize(t.after) == hipSuccess;
      if (ok) std::memcpy(t.pc.dst, t.pc.src, t.pc.bytes);
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (!ok) failed_[t.job] = 1;
        --left_[t.job];
      }
      done_cv_.notify_all();
    }
  }
  int device_;
  std::vector<size_t> left_;  // tasks outstanding per job
  std::vector<char> failed_;
  std::deque<Task> q_;
  bool stop_ = false;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> th_;
};

// Host threads that stage pageable inputs; XEC_PIPELINE_COPY_THREADS at
// xec_pipeline_create overrides (0 = none: HIP stages them, the old path).
constexpr unsigned kStageThreads = 4;
unsigned stage_threads() {
  const char* e = std::getenv("XEC_PIPELINE_COPY_THREADS");
  if (e == nullptr || *e == '\0') return kStageThreads;
  const long v = std::strtol(e, nullptr, 10);
  return v < 0 ? 0u : v > 32 ? 32u : (unsigned)v;
}

}  // namespace

struct xec_pipeline {
  int device = 0;
  size_t chunk_stripes = 0, bs = 0, k = 0, m = 0;
  struct Slot {
    hipStream_t stream = nullptr;
    uint8_t* data = nullptr;
    uint8_t* parity = nullptr;
    uint8_t* bitmap = nullptr;
    // pageable destinations only: chunk_stripes*m*bs pinned bytes (a chunk's
    // parity, or its rebuilt blocks -- at most m per stripe) and the event
    // after the D2H copies into them
    uint8_t* bounce = nullptr;
    hipEvent_t out_done = nullptr;
    // staged inputs only: a second stream the H2D copies alternate onto, the
    // event that frees the slot to it and the one the slot's stream joins
    hipStream_t aux = nullptr;
    hipEvent_t free_ev = nullptr, aux_done = nullptr;
  };
  std::vector<Slot> slots;
  HostCopier* copier = nullptr;  // made on the first pageable destination
  // pageable inputs: two pinned buffers laid out as a slot (data, then
  // parity), each with the event after the DMA that reads it
  unsigned stage_threads = 0;
  // XEC_PIPELINE_STAGE_OPTS (A/B): 'a' alternate H2D streams, 'f' first
  // chunk direct, 'm' main thread waits for the buffer, 'e' stage encode data
  // (a fuzz sequence that ended in a device error with 'a' -- profiles/r04q,
  // r04r -- turned out to be the library's buffer events on destroyed caller
  // streams, csrc/xec_api.cpp record_after; 300 fuzz cases pass since, r04u)
  bool opt_aux = true, opt_first = true, opt_main = false, opt_encode = true;
  bool opt_pinned_aux = false;  // 'p' (A/B): pinned inputs alternate over the two streams too
  // Serial inputs: each chunk's H2D copies start only after the previous
  // chunk's are done (one input transfer in flight at a time).  Measured
  // (tools/pageable_probe.py, profiles/r04m/staging_default.json, 3 rounds):
  // encode from pinned data +2 % (53.2 -> 54.3 GB/s; +3.8 % with pageable
  // parity out), but decode -6 % and encode from pageable data -3 %, so by
  // default only the encode from pinned data runs serial.  's' / 'n' in
  // XEC_PIPELINE_STAGE_OPTS force it on / off everywhere (A/B).
  int opt_serial = -1;  // -1 automatic, 0 never, 1 always
  hipEvent_t in_done = nullptr;
  bool in_recorded = false;
  struct Stage {
    uint8_t* host = nullptr;
    hipEvent_t read = nullptr;
    bool recorded = false;
  };
  static constexpr size_t kMaxStage = 4;
  Stage stage[kMaxStage];
  size_t stage_buffers = 2;  // in use (opts digit 2..4, A/B)
  HostPool* pool = nullptr;  // made on the first pageable source
};

namespace {

void destroy_slots(xec_pipeline* p) {
  for (auto& s : p->slots)
    if (s.stream) (void)hipStreamSynchronize(s.stream);
  delete p->copier;  // drains its queue: nothing reads a bounce buffer after this
  p->copier = nullptr;
  delete p->pool;  // likewise for the staging buffers
  p->pool = nullptr;
  for (auto& st : p->stage) {
    (void)hipHostFree(st.host);
    if (st.read) (void)hipEventDestroy(st.read);
    st = xec_pipeline::Stage{};
  }
  for (auto& s : p->slots) {
    (void)hipFree(s.data);
    (void)hipFree(s.parity);
    (void)hipFree(s.bitmap);
    (void)hipHostFree(s.bounce);
    if (s.out_done) (void)hipEventDestroy(s.out_done);
    if (s.free_ev) (void)hipEventDestroy(s.free_ev);
    if (s.aux_done) (void)hipEventDestroy(s.aux_done);
    if (s.aux) {
      (void)hipStreamSynchronize(s.aux);
      (void)hipStreamDestroy(s.aux);
    }
    if (s.stream) (void)hipStreamDestroy(s.stream);
  }
  p->slots.clear();
  if (p->in_done) (void)hipEventDestroy(p->in_done);
  p->in_done = nullptr;
}

// Whether the host buffer at q is pinned (page-locked and known to HIP).
// Pageable memory is not registered and hipPointerGetAttributes fails on it;
// that error -- ours -- is cleared so it cannot surface in a later
// hipGetLastError.  An error the caller has not read yet stays the caller's:
// with one pending the query is skipped and the buffer is treated as pageable
// (the bounce path, correct for any host memory), so nothing is cleared.
bool host_pinned(const void* q) {
  if (hipPeekAtLastError() != hipSuccess) return false;
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, q) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// Bounce buffers, their events and the helper thread, for results bound for
// pageable memory; false if any of them cannot be had.
bool ensure_bounce(xec_pipeline* p) {
  const size_t bytes = p->chunk_stripes * p->m * p->bs;
  for (auto& s : p->slots) {
    if (s.bounce == nullptr &&
        hipHostMalloc(reinterpret_cast<void**>(&s.bounce), bytes, hipHostMallocDefault) !=
            hipSuccess) {
      s.bounce = nullptr;
      return false;
    }
    if (s.out_done == nullptr &&
        hipEventCreateWithFlags(&s.out_done, hipEventDisableTiming) != hipSuccess) {
      s.out_done = nullptr;
      return false;
    }
  }
  if (p->copier == nullptr) {
    try {  // no exception crosses the C ABI (a thread may fail to start)
      p->copier = new HostCopier(p->device, p->slots.size());
    } catch (...) {
      p->copier = nullptr;
    }
  }
  return p->copier != nullptr;
}

// Each slot's second stream for input copies and its two events.
bool ensure_aux(xec_pipeline* p) {
  for (auto& s : p->slots) {
    if (s.aux == nullptr && hipStreamCreateWithFlags(&s.aux, hipStreamNonBlocking) != hipSuccess) {
      s.aux = nullptr;
      return false;
    }
    for (hipEvent_t* e : {&s.free_ev, &s.aux_done})
      if (*e == nullptr && hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) {
        *e = nullptr;
        return false;
      }
  }
  return true;
}

// Staging buffers, their events and the pool, for inputs from pageable
// memory; false if any of them cannot be had (or staging is off).
bool ensure_stage(xec_pipeline* p) {
  if (p->stage_threads == 0) return false;
  const size_t bytes = p->chunk_stripes * (p->k + p->m) * p->bs;
  for (size_t b = 0; b < p->stage_buffers; ++b) {
    auto& st = p->stage[b];
    if (st.host == nullptr &&
        hipHostMalloc(reinterpret_cast<void**>(&st.host), bytes, hipHostMallocDefault) !=
            hipSuccess) {
      st.host = nullptr;
      return false;
    }
    if (st.read == nullptr && hipEventCreateWithFlags(&st.read, hipEventDisableTiming) != hipSuccess) {
      st.read = nullptr;
      return false;
    }
  }
  if (p->opt_aux && !ensure_aux(p)) return false;
  if (p->pool == nullptr) {
    try {  // no exception crosses the C ABI (a thread may fail to start)
      p->pool = new HostPool(p->device, p->stage_threads, p->stage_buffers);
    } catch (...) {
      p->pool = nullptr;
    }
  }
  return p->pool != nullptr;
}

// Every queued copy done, the helper's host copies included.
xec_status sync_all(xec_pipeline* p) {
  xec_status st = XEC_SUCCESS;
  if (p->pool) p->pool->drain();  // no staging thread reads the caller's memory after this
  for (auto& s : p->slots)
    if (hipStreamSynchronize(s.stream) != hipSuccess ||
        (s.aux && hipStreamSynchronize(s.aux) != hipSuccess))
      st = XEC_DEVICE_ERROR;
  if (p->copier && !p->copier->drain()) st = XEC_DEVICE_ERROR;
  return st;
}

// The pipeline's streams and slots belong to the device current at create;
// each call runs there and gives the caller's current device back.
struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    ok = hipGetDevice(&prev) == hipSuccess && (prev == dev || hipSetDevice(dev) == hipSuccess);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (ok && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Error exit: drain what was already queued so no copy touches the caller's
// buffers after the call returns.
// XEC_PIPELINE_DEBUG=1: a failed call names its line and the HIP error
// pending at that point on stderr (diagnostics only).
bool debug_on() {
  static const bool on = [] {
    const char* e = std::getenv("XEC_PIPELINE_DEBUG");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

xec_status fail_at(xec_pipeline* p, xec_status st, int line) {
  if (debug_on())
    std::fprintf(stderr, "xec_pipeline: status %d at xec_pipeline.cpp:%d, pending HIP error %s\n",
                 (int)st, line, hipGetErrorName(hipPeekAtLastError()));
  (void)sync_all(p);
  return st;
}
#define fail(p, st) fail_at((p), (st), __LINE__)

// Copy runs of consecutive indices i < n with want(i) -- adjacent blocks merge
// into one copy.
template <typename W, typename F>
bool for_runs(size_t n, W&& want, F&& copy) {
  size_t i = 0;
  while (i < n) {
    if (!want(i)) {
      ++i;
      continue;
    }
    size_t j = i;
    while (j < n && want(j)) ++j;
    if (!copy(i, j)) return false;
    i = j;
  }
  return true;
}

// Blocks from this size on travel only where a rebuild reads them (the
// members and parity of classes that lost a data block); smaller blocks
// travel as whole runs of survivors, where one copy per block would cost more
// in per-copy overhead than the bytes it saves.  With m = 1 both are the same.
constexpr size_t kSelectiveCopyBytes = 64u << 10;

// Below this block size a decode's copies are counted, not its bytes: every
// H2D / D2H command costs ~10 us of SDMA start-up, while the
// bytes a per-run copy would save -- the lost blocks' -- move in 1/k of a
// chunk's time.  So a chunk's (non-selective) inputs go up whole and its
// rebuilt blocks are gathered on the device and come back as one copy
// (profiles/r05j, r05k: config 4's shape 12.8 -> 52.1 GB/s pinned, 15.5 ->
// 53.4 pageable).  At 1 MiB blocks per-run copies tie whole ones and save the
// lost blocks' PCIe bytes, so they stay (config 3: 55 GB/s, the PCIe bound).
constexpr size_t kWholeCopyBelowBytes = 1u << 20;

// A chunk's outputs (parity, or rebuilt blocks) are queued after the next
// chunk's inputs rather than right behind its own kernel, so the copy engine
// has the next chunk's input queued before the host waits on anything.
// Measured: pinned encode +2.3 % (52.8 -> 54.0 GB/s at config 3, 8-stripe
// chunks x 3 streams, tools/pageable_probe.py, profiles/r03q).
constexpr bool kDeferOutputs = true;

// One H2D copy of a chunk's inputs: `bytes` from host `src` to `off` bytes
// into the slot's data region (or, `parity`, its parity region).
struct InRun {
  bool parity;
  size_t off;
  const uint8_t* src;
  size_t bytes;
};

// A chunk's inputs, staged or not.  Staged runs (source in pageable memory)
// are first copied by the pool into staging buffer `chunk_no % nb_` at the
// slot's offsets (`prefetch`, while the previous chunk's DMA runs); `issue`
// then queues every run on the slot's stream -- staged ones from the staging
// buffer, the rest straight from the caller's pinned memory -- and marks the
// buffer read once the stream has passed its copies.
class Inputs {
 public:
  // `serial_auto`: whether the caller's inputs run serial when the pipeline's
  // option is automatic
  Inputs(xec_pipeline* p, bool stage_data, bool stage_parity, bool serial_auto = false)
      : p_(p), sd_(stage_data), sp_(stage_parity),
        serial_(p->opt_serial < 0 ? serial_auto : p->opt_serial == 1),
        parity_at_(p->chunk_stripes * p->k * p->bs), nb_(p->stage_buffers) {
    p->in_recorded = false;  // a new call: nothing of its own to wait for yet
  }
  bool staged() const { return sd_ || sp_; }
  // how many chunks ahead the pool stages: one per staging buffer but the
  // one the DMA is reading
  size_t ahead() const { return staged() ? nb_ - 1 : 0; }
  template <typename Runs>
  void prefetch(size_t chunk_no, Runs&& runs) {
    if (!staged()) return;
    auto& st = p_->stage[chunk_no % nb_];
    std::vector<HostPool::Piece> pieces;
    runs([&](const InRun& r) {
      if (r.parity ? sp_ : sd_)
        pieces.push_back({st.host + (r.parity ? parity_at_ : 0) + r.off, r.src, r.bytes});
      return true;
    });
    hipEvent_t after = st.recorded ? st.read : nullptr;
    failed_[chunk_no % nb_] = false;
    if (after != nullptr && p_->opt_main) {
      if (hipEventSynchronize(after) != hipSuccess) {  // issue() then fails
        pieces.clear();
        failed_[chunk_no % nb_] = true;
      }
      after = nullptr;
    }
    p_->pool->submit(chunk_no % nb_, after, pieces);
  }
  // `direct`: this chunk's runs all read the caller's memory on the slot's
  // stream (HIP stages pageable ones) -- the first chunk of a call, so that
  // its DMA starts at once while the pool stages the next one.
  template <typename Runs>
  bool issue(size_t chunk_no, xec_pipeline::Slot& s, Runs&& runs, bool direct = false) {
    if (!serial_ || p_->in_done == nullptr) return issue_impl(chunk_no, s, runs, direct);
    if (p_->in_recorded && hipStreamWaitEvent(s.stream, p_->in_done, 0) != hipSuccess) return false;
    if (!issue_impl(chunk_no, s, runs, direct)) return false;
    p_->in_recorded = hipEventRecord(p_->in_done, s.stream) == hipSuccess;
    return p_->in_recorded;
  }

 private:
  template <typename Runs>
  bool issue_impl(size_t chunk_no, xec_pipeline::Slot& s, Runs&& runs, bool direct) {
    if (!staged() || direct) {
      if (!staged() && p_->opt_pinned_aux && s.aux != nullptr)  // 'p': pinned inputs alternate
        return alternate(s, runs, [](const InRun& r) { return r.src; });
      return runs([&](const InRun& r) {
        return hipMemcpyAsync((r.parity ? s.parity : s.data) + r.off, r.src, r.bytes,
                              hipMemcpyHostToDevice, s.stream) == hipSuccess;
      });
    }
    auto& st = p_->stage[chunk_no % nb_];
    if (!p_->pool->wait(chunk_no % nb_) || failed_[chunk_no % nb_]) return false;
    const bool ok = alternate(s, runs, [&](const InRun& r) {
      return (r.parity ? sp_ : sd_) ? st.host + (r.parity ? parity_at_ : 0) + r.off : r.src;
    });
    if (ok && hipEventRecord(st.read, s.stream) == hipSuccess) {
      st.recorded = true;
      return true;
    }
    if (s.aux) (void)hipStreamSynchronize(s.aux);  // nothing reads the buffer after this
    (void)hipStreamSynchronize(s.stream);
    st.recorded = false;
    return false;
  }

  // The runs alternate between the slot's stream and its aux stream (when it
  // has one), so one copy's start-up hides behind the other's transfer; aux
  // first waits until the slot's stream is done with the slot's previous
  // chunk, and the slot's stream then waits for aux.  `src_of(run)`: where
  // the run's bytes are read from.
  template <typename Runs, typename Src>
  bool alternate(xec_pipeline::Slot& s, Runs&& runs, Src&& src_of) {
    hipStream_t other = s.aux != nullptr ? s.aux : s.stream;
    if (other != s.stream && (hipEventRecord(s.free_ev, s.stream) != hipSuccess ||
                              hipStreamWaitEvent(other, s.free_ev, 0) != hipSuccess)) {
      if (debug_on()) std::fprintf(stderr, "xec_pipeline: aux wait failed\n");
      return false;
    }
    size_t n = 0;
    bool ok = runs([&](const InRun& r) {
      const hipError_t e = hipMemcpyAsync((r.parity ? s.parity : s.data) + r.off, src_of(r),
                                          r.bytes, hipMemcpyHostToDevice,
                                          (n++ % 2) ? other : s.stream);
      if (e != hipSuccess && debug_on())
        std::fprintf(stderr, "xec_pipeline: H2D of %zu bytes (run %zu) failed: %s\n", r.bytes,
                     n - 1, hipGetErrorName(e));
      return e == hipSuccess;
    });
    if (other != s.stream)
      ok = (hipEventRecord(s.aux_done, other) == hipSuccess &&
            hipStreamWaitEvent(s.stream, s.aux_done, 0) == hipSuccess) && ok;
    return ok;
  }

  xec_pipeline* p_;
  bool sd_, sp_, serial_;
  size_t parity_at_;
  size_t nb_;
  bool failed_[xec_pipeline::kMaxStage] = {};
};

}  // namespace

extern "C" {

static xec_status create_impl(xec_pipeline** out, size_t chunk_stripes, size_t bs, size_t k,
                               size_t m, int nstreams) {
  if (!out) return XEC_INVALID_SIZE;
  *out = nullptr;
  // the pipeline's device slots are 64-B aligned by hipMalloc; check the rest
  xec_status st = xec_check_args(reinterpret_cast<void*>(64), reinterpret_cast<void*>(64), bs, k, m);
  if (st != XEC_SUCCESS) return st;
  if (chunk_stripes == 0 || nstreams < 1 || nstreams > 16) return XEC_INVALID_SIZE;
  // a slot's chunk_stripes*(k+m)*bs bytes must be representable (k, m and bs
  // are bounded by the checks above only from below)
  const size_t row_bytes = (k + m) * bs;
  if (k + m < k || row_bytes / bs != k + m || chunk_stripes > SIZE_MAX / row_bytes)
    return XEC_INVALID_SIZE;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return XEC_DEVICE_ERROR;
  auto* p = new (std::nothrow) xec_pipeline;
  if (!p) return XEC_DEVICE_ERROR;
  p->device = dev;
  p->stage_threads = stage_threads();
  if (const char* e = std::getenv("XEC_PIPELINE_STAGE_OPTS")) {
    const std::string o(e);
    p->opt_aux = o.find('a') != std::string::npos;
    p->opt_first = o.find('f') != std::string::npos;
    p->opt_main = o.find('m') != std::string::npos;
    p->opt_encode = o.find('e') != std::string::npos;
    p->opt_pinned_aux = o.find('p') != std::string::npos;
    p->opt_serial = o.find('s') != std::string::npos ? 1 : o.find('n') != std::string::npos ? 0 : -1;
    for (char c : o)
      if (c >= '2' && c <= '4') p->stage_buffers = (size_t)(c - '0');
  }
  p->chunk_stripes = chunk_stripes;
  p->bs = bs;
  p->k = k;
  p->m = m;
  p->slots.resize(static_cast<size_t>(nstreams));
  if (p->opt_serial != 0 && hipEventCreateWithFlags(&p->in_done, hipEventDisableTiming) != hipSuccess)
    p->in_done = nullptr;  // then inputs are never serialised
  for (auto& s : p->slots) {
    if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&s.data, chunk_stripes * k * bs) != hipSuccess ||
        hipMalloc(&s.parity, chunk_stripes * m * bs) != hipSuccess ||
        hipMalloc(&s.bitmap, chunk_stripes * (k + m)) != hipSuccess) {
      destroy_slots(p);
      delete p;
      return XEC_DEVICE_ERROR;
    }
  }
  *out = p;
  return XEC_SUCCESS;
}

xec_status xec_pipeline_destroy(xec_pipeline* p) {
  if (!p) return XEC_SUCCESS;
  const DeviceGuard dg(p->device);
  destroy_slots(p);
  delete p;
  return XEC_SUCCESS;
}

static xec_status encode_impl(xec_pipeline* p, const void* h_data, void* h_parity, size_t S) {
  if (!p) return XEC_NOT_INITIALIZED;
  const DeviceGuard dg(p->device);
  if (!dg.ok) return XEC_DEVICE_ERROR;
  const size_t k = p->k, m = p->m, bs = p->bs, cs = p->chunk_stripes;
  const auto* src = static_cast<const uint8_t*>(h_data);
  auto* dst = static_cast<uint8_t*>(h_parity);
  const size_t ns = p->slots.size();
  // a chunk's parity copy-out is queued after the NEXT chunk's input (see
  // kDeferOutputs); with one slot the next chunk would overwrite it first
  const bool defer = kDeferOutputs && ns > 1;
  // parity bound for pageable memory leaves through the bounce buffers, data
  // from pageable memory comes in through the staging buffers
  const bool bounce = S > 0 && !host_pinned(h_parity);
  if (bounce && !ensure_bounce(p)) return XEC_DEVICE_ERROR;
  const bool data_pinned = S == 0 || host_pinned(h_data);
  Inputs in(p, p->opt_encode && !data_pinned && ensure_stage(p), false, data_pinned);
  auto out = [&](size_t chunk) {
    const size_t c0 = chunk * cs, n = (S - c0) < cs ? (S - c0) : cs;
    const size_t si = chunk % ns;
    auto& s = p->slots[si];
    if (!bounce)
      return hipMemcpyAsync(dst + c0 * m * bs, s.parity, n * m * bs, hipMemcpyDeviceToHost,
                            s.stream) == hipSuccess;
    p->copier->wait_slot(si);
    if (hipMemcpyAsync(s.bounce, s.parity, n * m * bs, hipMemcpyDeviceToHost, s.stream) !=
            hipSuccess ||
        hipEventRecord(s.out_done, s.stream) != hipSuccess)
      return false;
    p->copier->push(si, s.out_done, {{dst + c0 * m * bs, s.bounce, n * m * bs}});
    return true;
  };
  auto runs = [&](size_t chunk) {
    return [&, chunk](auto&& f) {
      const size_t c0 = chunk * cs, n = (S - c0) < cs ? (S - c0) : cs;
      return f(InRun{false, 0, src + c0 * k * bs, n * k * bs});
    };
  };
  const size_t chunks = (S + cs - 1) / cs;
  // the first chunk comes in directly (opt_first) while the pool stages the next
  const size_t first = in.staged() && p->opt_first ? 1 : 0;
  for (size_t q = first; q < chunks && q < first + in.ahead(); ++q) in.prefetch(q, runs(q));
  for (size_t chunk = 0; chunk < chunks; ++chunk) {
    const size_t n = (S - chunk * cs) < cs ? (S - chunk * cs) : cs;
    auto& s = p->slots[chunk % ns];
    // stream order serialises reuse of this slot behind its previous chunk
    if (!in.issue(chunk, s, runs(chunk), chunk < first)) return fail(p, XEC_DEVICE_ERROR);
    const size_t next = chunk + in.ahead();
    if (chunk >= first && next < chunks) in.prefetch(next, runs(next));
    xec_status st = xec_encode(s.data, s.parity, n, bs, k, m, s.stream);
    if (st != XEC_SUCCESS) return fail(p, st);
    if (defer ? (chunk > 0 && !out(chunk - 1)) : !out(chunk)) return fail(p, XEC_DEVICE_ERROR);
  }
  if (defer && chunks > 0 && !out(chunks - 1)) return fail(p, XEC_DEVICE_ERROR);
  return sync_all(p);
}

static xec_status decode_impl(xec_pipeline* p, void* h_data, const void* h_parity, size_t S,
                               const uint8_t* h_bitmap) {
  if (!p) return XEC_NOT_INITIALIZED;
  const DeviceGuard dg(p->device);
  if (!dg.ok) return XEC_DEVICE_ERROR;
  const size_t k = p->k, m = p->m, bs = p->bs, row = k + m, cs = p->chunk_stripes;
  int needs = 0;
  xec_status st = xec_check_bitmap(h_bitmap, S, k, m, &needs);
  if (st != XEC_SUCCESS || !needs) return st;  // all-or-nothing, as xec_decode
  auto* data = static_cast<uint8_t*>(h_data);
  const auto* par = static_cast<const uint8_t*>(h_parity);
  const bool selective = m > 1 && bs >= kSelectiveCopyBytes;
  const size_t ns = p->slots.size();
  const bool defer = kDeferOutputs && ns > 1;  // as in xec_pipeline_encode
  // Pageable h_data: the rebuilt blocks leave through the bounce buffers.
  // Pageable inputs come in through the staging buffers; when staging is off
  // (or cannot be had) every copy from pageable h_data holds this thread until
  // done, so a chunk's data then comes in as ONE copy, lost blocks included
  // (their content is never read), instead of one copy per run of survivors
  // -- ~20 us of host time per call, against the 1/k more bytes (profiles/r03v).
  const bool pageable = !host_pinned(h_data);
  const bool paged_parity = !host_pinned(h_parity);
  // Below kWholeCopyBelowBytes one copy per run of survivors in and one per
  // rebuilt block out cost more than the bytes (config 4's shape: pinned
  // decode 12.8 GB/s, config 2's 30; tools/pageable_probe.py, profiles/r05j,
  // r05k).  So there a chunk's non-selective inputs go up whole (pinned or
  // staged), and its rebuilt blocks are gathered on the device into the
  // slot's parity region -- free once the decode kernel has read it -- and
  // leave as ONE D2H copy into the slot's bounce buffer, which the helper
  // thread scatters (u32 items c << 8 | i: k <= 256, fewer than 2^24 stripes
  // per chunk).
  const bool gather = bs < kWholeCopyBelowBytes && k <= 256 && cs <= (size_t{1} << 24);
  if ((pageable || gather) && !ensure_bounce(p)) return XEC_DEVICE_ERROR;
  const bool stage = (pageable || paged_parity) && ensure_stage(p);
  if (!stage && p->opt_pinned_aux) (void)ensure_aux(p);  // without: one stream, as before
  Inputs in(p, stage && pageable, stage && paged_parity);
  // (the first chunk of a staged call comes in directly, so whole too)
  const bool whole_direct = (pageable || bs < kWholeCopyBelowBytes) && !selective;
  // Staged, the pool copies each run into the staging buffer at the slot's
  // offsets and every run then goes up as its own copy: with large blocks
  // that saves the lost blocks' PCIe bytes (1/k of a PCIe-bound leg); with
  // smaller ones (config 4: k=32+1 x 4 KiB, two runs per stripe) the
  // per-copy cost would dominate, so below kWholeCopyBelowBytes the whole
  // chunk is staged and goes up as one copy, as unstaged.
  const bool whole_chunks = whole_direct && (!stage || bs < kWholeCopyBelowBytes);
  // D2H of the rebuilt blocks of `chunk` (only those: a survivor's bytes are
  // already in the caller's buffer)
  auto gather_out = [&](size_t chunk, size_t slot) {
    const size_t c0 = chunk * cs, n = (S - c0) < cs ? (S - c0) : cs;
    auto& s = p->slots[slot];
    p->copier->wait_slot(slot);
    std::vector<uint32_t> items;
    std::vector<HostCopier::Piece> owed;
    for (size_t c = c0; c < c0 + n; ++c)
      for (size_t i = 0; i < k; ++i)
        if (h_bitmap[c * row + i] == 0) {
          owed.push_back({data + (c * k + i) * bs, s.bounce + items.size() * bs, bs});
          items.push_back(static_cast<uint32_t>(((c - c0) << 8) | i));
        }
    for (size_t g0 = 0; g0 < items.size(); g0 += xec::kArgItems) {
      const size_t g = items.size() - g0 < xec::kArgItems ? items.size() - g0 : xec::kArgItems;
      if (xec::launch_gather(s.data, s.parity + g0 * bs, k, bs, items.data() + g0, g, s.stream) !=
          hipSuccess)
        return false;
    }
    if (hipMemcpyAsync(s.bounce, s.parity, items.size() * bs, hipMemcpyDeviceToHost, s.stream) !=
            hipSuccess ||
        hipEventRecord(s.out_done, s.stream) != hipSuccess)
      return false;
    p->copier->push(slot, s.out_done, std::move(owed));
    return true;
  };
  auto out = [&](size_t chunk, size_t slot) {
    if (gather) return gather_out(chunk, slot);
    const size_t c0 = chunk * cs, n = (S - c0) < cs ? (S - c0) : cs;
    auto& s = p->slots[slot];
    std::vector<HostCopier::Piece> owed;
    size_t off = 0;  // bounce offset: at most m rebuilt blocks per stripe
    if (pageable) p->copier->wait_slot(slot);
    for (size_t c = c0; c < c0 + n; ++c) {
      const uint8_t* bm = h_bitmap + c * row;
      const size_t base = c * k * bs, sbase = (c - c0) * k * bs;
      if (!for_runs(k, [&](size_t i) { return bm[i] == 0; }, [&](size_t i, size_t j) {
            const size_t bytes = (j - i) * bs;
            uint8_t* to = data + base + i * bs;
            if (pageable) {
              owed.push_back({to, s.bounce + off, bytes});
              to = s.bounce + off;
              off += bytes;
            }
            return hipMemcpyAsync(to, s.data + sbase + i * bs, bytes, hipMemcpyDeviceToHost,
                                  s.stream) == hipSuccess;
          }))
        return false;
    }
    if (pageable) {
      if (hipEventRecord(s.out_done, s.stream) != hipSuccess) return false;
      p->copier->push(slot, s.out_done, std::move(owed));
    }
    return true;
  };
  // H2D: the surviving data blocks a rebuild reads (a lost block's content is
  // never read) and the parity; D2H: only the rebuilt blocks.  With selective
  // copies only the classes that lost a data block travel (xorec.cpp:79-108
  // reads nothing else).
  auto runs = [&](size_t chunk, bool whole) {
    return [&, chunk, whole](auto&& f) -> bool {
      const size_t c0 = chunk * cs, n = (S - c0) < cs ? (S - c0) : cs;
      if (whole && !f(InRun{false, 0, data + c0 * k * bs, n * k * bs})) return false;
      std::vector<uint8_t> class_lost(m);
      for (size_t c = c0; c < c0 + n && !whole; ++c) {
        const uint8_t* bm = h_bitmap + c * row;
        const size_t base = c * k * bs, sbase = (c - c0) * k * bs, pbase = (c - c0) * m * bs;
        for (size_t j = 0; j < m; ++j) class_lost[j] = 0;
        for (size_t i = 0; i < k; ++i)
          if (bm[i] == 0) class_lost[i % m] = 1;
        if (!for_runs(k, [&](size_t i) { return bm[i] != 0 && (!selective || class_lost[i % m]); },
                      [&](size_t i, size_t j) {
                        return f(InRun{false, sbase + i * bs, data + base + i * bs, (j - i) * bs});
                      }) ||
            (selective && !for_runs(m, [&](size_t j) { return class_lost[j] != 0; },
                                    [&](size_t i, size_t j) {
                                      return f(InRun{true, pbase + i * bs, par + c * m * bs + i * bs,
                                                     (j - i) * bs});
                                    })))
          return false;
      }
      return selective || f(InRun{true, 0, par + c0 * m * bs, n * m * bs});
    };
  };
  // The chunks that rebuild something (a chunk without a loss moves nothing).
  // Slots go round them, so consecutive rebuilding chunks never share a slot.
  std::vector<size_t> work;
  for (size_t c0 = 0, chunk = 0; c0 < S; c0 += cs, ++chunk) {
    const size_t n = (S - c0) < cs ? (S - c0) : cs;
    bool any_lost = false;
    for (size_t c = c0; c < c0 + n && !any_lost; ++c)
      for (size_t i = 0; i < k; ++i)
        if (h_bitmap[c * row + i] == 0) {
          any_lost = true;
          break;
        }
    if (any_lost) work.push_back(chunk);
  }
  size_t pending = 0, pending_slot = 0;
  bool have_pending = false;
  // the first rebuilding chunk comes in directly (opt_first) while the pool
  // stages the next
  const size_t first = in.staged() && p->opt_first ? 1 : 0;
  for (size_t q = first; q < work.size() && q < first + in.ahead(); ++q)
    in.prefetch(q, runs(work[q], whole_chunks));
  for (size_t u = 0; u < work.size(); ++u) {
    const size_t chunk = work[u], c0 = chunk * cs, n = (S - c0) < cs ? (S - c0) : cs;
    const size_t slot = u % ns;
    auto& s = p->slots[slot];
    const bool direct = u < first;
    if (!in.issue(u, s, runs(chunk, direct ? whole_direct : whole_chunks), direct))
      return fail(p, XEC_DEVICE_ERROR);
    const size_t next = u + in.ahead();
    if (u >= first && next < work.size()) in.prefetch(next, runs(work[next], whole_chunks));
    st = xec_decode(s.data, s.parity, n, bs, k, m, h_bitmap + c0 * row, s.bitmap, s.stream);
    if (st != XEC_SUCCESS) return fail(p, st);
    if (!defer) {
      if (!out(chunk, slot)) return fail(p, XEC_DEVICE_ERROR);
      continue;
    }
    // the previous rebuilding chunk's outputs go behind this chunk's inputs
    // (another slot); its own slot takes new inputs only ns >= 2 rebuilding
    // chunks later, after these outputs are queued on its stream
    if (have_pending && !out(pending, pending_slot)) return fail(p, XEC_DEVICE_ERROR);
    pending = chunk;
    pending_slot = slot;
    have_pending = true;
  }
  if (have_pending && !out(pending, pending_slot)) return fail(p, XEC_DEVICE_ERROR);
  return sync_all(p);
}

// No exception crosses the C ABI: the host bookkeeping allocates (slots, run
// lists, the helper thread), and a failure there is a device error for the
// caller.  Whatever was queued is drained first, so nothing touches the
// caller's buffers after the call returns.
xec_status xec_pipeline_create(xec_pipeline** out, size_t chunk_stripes, size_t bs, size_t k,
                               size_t m, int nstreams) {
  try {
    return create_impl(out, chunk_stripes, bs, k, m, nstreams);
  } catch (...) {
    return XEC_DEVICE_ERROR;
  }
}

xec_status xec_pipeline_encode(xec_pipeline* p, const void* h_data, void* h_parity, size_t S) {
  xec::t_kernel_events = xec::KernelEvents{};  // xec_set_kernel_events is not for the pipeline
  try {
    return encode_impl(p, h_data, h_parity, S);
  } catch (...) {
    return p ? fail(p, XEC_DEVICE_ERROR) : XEC_DEVICE_ERROR;
  }
}

xec_status xec_pipeline_decode(xec_pipeline* p, void* h_data, const void* h_parity, size_t S,
                               const uint8_t* h_bitmap) {
  xec::t_kernel_events = xec::KernelEvents{};  // xec_set_kernel_events is not for the pipeline
  try {
    return decode_impl(p, h_data, h_parity, S, h_bitmap);
  } catch (...) {
    return p ? fail(p, XEC_DEVICE_ERROR) : XEC_DEVICE_ERROR;
  }
}

}  // extern "C"
