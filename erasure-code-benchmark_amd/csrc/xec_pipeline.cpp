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

#include <new>
#include <vector>

#include "xec.h"
#include "xec_kernels.h"

struct xec_pipeline {
  int device = 0;
  size_t chunk_stripes = 0, bs = 0, k = 0, m = 0;
  struct Slot {
    hipStream_t stream = nullptr;
    uint8_t* data = nullptr;
    uint8_t* parity = nullptr;
    uint8_t* bitmap = nullptr;
  };
  std::vector<Slot> slots;
};

namespace {

void destroy_slots(xec_pipeline* p) {
  for (auto& s : p->slots) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    (void)hipFree(s.data);
    (void)hipFree(s.parity);
    (void)hipFree(s.bitmap);
    if (s.stream) (void)hipStreamDestroy(s.stream);
  }
  p->slots.clear();
}

xec_status sync_all(xec_pipeline* p) {
  xec_status st = XEC_SUCCESS;
  for (auto& s : p->slots)
    if (hipStreamSynchronize(s.stream) != hipSuccess) st = XEC_DEVICE_ERROR;
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
xec_status fail(xec_pipeline* p, xec_status st) {
  (void)sync_all(p);
  return st;
}

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

// A chunk's outputs (parity, or rebuilt blocks) are queued after the next
// chunk's inputs rather than right behind its own kernel, so the copy engine
// has the next chunk's input queued before the host waits on anything
// (tools/pageable_probe.py).  Measured: pinned encode +2.3 % (52.8 -> 54.0
// GB/s at config 3, 8-stripe chunks x 3 streams, profiles/r03q), decode and
// the pageable rates unchanged.
constexpr bool kDeferOutputs = true;

}  // namespace

extern "C" {

xec_status xec_pipeline_create(xec_pipeline** out, size_t chunk_stripes, size_t bs, size_t k,
                               size_t m, int nstreams) {
  if (!out) return XEC_INVALID_SIZE;
  *out = nullptr;
  // the pipeline's device slots are 64-B aligned by hipMalloc; check the rest
  xec_status st = xec_check_args(reinterpret_cast<void*>(64), reinterpret_cast<void*>(64), bs, k, m);
  if (st != XEC_SUCCESS) return st;
  if (chunk_stripes == 0 || nstreams < 1 || nstreams > 16) return XEC_INVALID_SIZE;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return XEC_DEVICE_ERROR;
  auto* p = new (std::nothrow) xec_pipeline;
  if (!p) return XEC_DEVICE_ERROR;
  p->device = dev;
  p->chunk_stripes = chunk_stripes;
  p->bs = bs;
  p->k = k;
  p->m = m;
  p->slots.resize(static_cast<size_t>(nstreams));
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

xec_status xec_pipeline_encode(xec_pipeline* p, const void* h_data, void* h_parity, size_t S) {
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
  auto out = [&](size_t chunk) {
    const size_t c0 = chunk * cs, n = (S - c0) < cs ? (S - c0) : cs;
    auto& s = p->slots[chunk % ns];
    return hipMemcpyAsync(dst + c0 * m * bs, s.parity, n * m * bs, hipMemcpyDeviceToHost,
                          s.stream) == hipSuccess;
  };
  size_t chunk = 0;
  for (size_t c0 = 0; c0 < S; c0 += cs, ++chunk) {
    auto& s = p->slots[chunk % ns];
    const size_t n = (S - c0) < cs ? (S - c0) : cs;
    // stream order serialises reuse of this slot behind its previous chunk
    if (hipMemcpyAsync(s.data, src + c0 * k * bs, n * k * bs, hipMemcpyHostToDevice, s.stream) !=
        hipSuccess)
      return fail(p, XEC_DEVICE_ERROR);
    xec_status st = xec_encode(s.data, s.parity, n, bs, k, m, s.stream);
    if (st != XEC_SUCCESS) return fail(p, st);
    if (defer ? (chunk > 0 && !out(chunk - 1)) : !out(chunk)) return fail(p, XEC_DEVICE_ERROR);
  }
  if (defer && chunk > 0 && !out(chunk - 1)) return fail(p, XEC_DEVICE_ERROR);
  return sync_all(p);
}

xec_status xec_pipeline_decode(xec_pipeline* p, void* h_data, const void* h_parity, size_t S,
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
  std::vector<uint8_t> class_lost(m);
  // D2H of the rebuilt blocks of `chunk` (only those: a survivor's bytes are
  // already in the caller's buffer)
  auto out = [&](size_t chunk, size_t slot) {
    const size_t c0 = chunk * cs, n = (S - c0) < cs ? (S - c0) : cs;
    auto& s = p->slots[slot];
    for (size_t c = c0; c < c0 + n; ++c) {
      const uint8_t* bm = h_bitmap + c * row;
      const size_t base = c * k * bs, sbase = (c - c0) * k * bs;
      if (!for_runs(k, [&](size_t i) { return bm[i] == 0; }, [&](size_t i, size_t j) {
            return hipMemcpyAsync(data + base + i * bs, s.data + sbase + i * bs, (j - i) * bs,
                                  hipMemcpyDeviceToHost, s.stream) == hipSuccess;
          }))
        return false;
    }
    return true;
  };
  // Slots go round the chunks that rebuild something (a chunk without a loss
  // moves nothing), so consecutive rebuilding chunks never share a slot.
  size_t chunk = 0, used = 0, pending = 0, pending_slot = 0;
  bool have_pending = false;
  for (size_t c0 = 0; c0 < S; c0 += cs, ++chunk) {
    const size_t n = (S - c0) < cs ? (S - c0) : cs;
    bool any_lost = false;
    for (size_t c = c0; c < c0 + n && !any_lost; ++c)
      for (size_t i = 0; i < k; ++i)
        if (h_bitmap[c * row + i] == 0) {
          any_lost = true;
          break;
        }
    if (!any_lost) continue;  // nothing of this chunk crosses the link
    const size_t slot = used++ % ns;
    auto& s = p->slots[slot];
    // H2D: the surviving data blocks a rebuild reads (a lost block's content
    // is never read) and the parity; D2H: only the rebuilt blocks.  With
    // selective copies only the classes that lost a data block travel
    // (xorec.cpp:79-108 reads nothing else).
    for (size_t c = c0; c < c0 + n; ++c) {
      const uint8_t* bm = h_bitmap + c * row;
      const size_t base = c * k * bs, sbase = (c - c0) * k * bs;
      for (size_t j = 0; j < m; ++j) class_lost[j] = 0;
      for (size_t i = 0; i < k; ++i)
        if (bm[i] == 0) class_lost[i % m] = 1;
      const auto h2d = [&](uint8_t* d, const uint8_t* h) {
        return [&, d, h](size_t i, size_t j) {
          return hipMemcpyAsync(d + i * bs, h + i * bs, (j - i) * bs, hipMemcpyHostToDevice,
                                s.stream) == hipSuccess;
        };
      };
      if (!for_runs(k, [&](size_t i) { return bm[i] != 0 && (!selective || class_lost[i % m]); },
                    h2d(s.data + sbase, data + base)) ||
          (selective && !for_runs(m, [&](size_t j) { return class_lost[j] != 0; },
                                  h2d(s.parity + (c - c0) * m * bs, par + c * m * bs))))
        return fail(p, XEC_DEVICE_ERROR);
    }
    if (!selective && hipMemcpyAsync(s.parity, par + c0 * m * bs, n * m * bs,
                                     hipMemcpyHostToDevice, s.stream) != hipSuccess)
      return fail(p, XEC_DEVICE_ERROR);
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

}  // extern "C"
