// xec_internal.h -- host-side helpers shared inside libxec_hip.so (plain C++,
// no HIP types, so xec_scan.cpp still builds without the HIP device pass).
// Not part of the public boundary (include/xec.h).
#pragma once

#include <cstddef>
#include <cstdint>

#include "xec.h"

// xec_check_bitmap plus the number of lost (zero) data bytes in the batch;
// lost_data may be null.  Defined in xec_scan.cpp.
xec_status xec_scan_bitmap(const uint8_t* h_bitmap, size_t S, size_t k, size_t m,
                           int* needs_recovery, uint64_t* lost_data);
