// xec_internal.h -- host-side helpers shared inside libxec_hip.so (plain C++,
// no HIP types, so xec_scan.cpp still builds without the HIP device pass).
// Not part of the public boundary (include/xec.h).
#pragma once

#include <cstddef>
#include <cstdint>

#include "xec.h"

// One decode work item: a lost data block, stripe c, block i (i < k <= 256,
// c < 2^24), packed as c << 8 | i (xec_kernels.hip decode_list_kernel).
constexpr size_t kWorkItemMaxK = 256;
constexpr size_t kWorkItemMaxStripes = size_t(1) << 24;
inline uint32_t xec_work_item(size_t c, size_t i) {
  return static_cast<uint32_t>(c << 8) | static_cast<uint32_t>(i);
}

// What one host pass over a batch bitmap finds (xec_scan_bitmap).
struct XecScan {
  int needs_recovery = 0;     // require_recovery over the batch (bit 0 of a data byte clear)
  uint64_t lost_data = 0;     // zero data bytes
  uint64_t stripes_lost = 0;  // stripes with at least one zero data byte
  int64_t lost_class = -1;    // the parity class every lost data block is in, or -1
                              // (none lost, or several classes): one failed device
  uint64_t listed = 0;        // work items written; the list is whole iff == lost_data
};

// xec_check_bitmap plus the counts above (out may be null) and, when `items`
// is non-null, the first `cap` lost data blocks as work items in batch order
// (requires k <= kWorkItemMaxK and S <= kWorkItemMaxStripes).  `speculative`:
// the caller may not need the list at all, so listing stops once the losses
// seen so far, projected over the batch, say it will not be used -- more than
// `cap` of them, or a batch dense enough for class tiles (lost > S and
// 2 * lost >= S * m, xec_api.cpp use_class_tiles) -- and out->listed tells how
// many were written.  Defined in xec_scan.cpp.
xec_status xec_scan_bitmap(const uint8_t* h_bitmap, size_t S, size_t k, size_t m, XecScan* out,
                           uint32_t* items, uint64_t cap, bool speculative = false);

// Per-stripe form (the reference CPU plugin's loop, xorec_bm.cpp:43-58 over
// xorec_decode, xorec.cpp:62-111): codes[c] (if non-null) = 0 or 4
// (DecodeFailure) for every stripe; *failures = stripes with 4; work items
// (first `cap` to `items`) and *n_items only for stripes that need recovery
// and are recoverable.  XEC_INVALID_COUNTS as xec_check_args, else success.
xec_status xec_scan_stripes(const uint8_t* h_bitmap, size_t S, size_t k, size_t m,
                            uint8_t* codes, uint32_t* items, uint64_t cap, uint64_t* n_items,
                            uint64_t* failures);

// masks[c] = bit i set iff data byte i of stripe c's row is 0 (lost), for the
// kernel-argument mask decode (xec_kernels.hip decode_argmask_kernel).
// Requires k <= 32; the rows must already have passed xec_scan_bitmap (no
// checks here).  Defined in xec_scan.cpp.
void xec_loss_masks(const uint8_t* h_bitmap, size_t S, size_t k, size_t m, uint32_t* masks);
