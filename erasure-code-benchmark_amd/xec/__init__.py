"""xec -- MI355X-native XOR-EC encode / single-erasure decode (Python view).

The hot path is libxec_hip.so (hand-written gfx950 HIP kernels behind the C ABI
of include/xec.h).  This package only binds it for tests, bench.py and the
multi-GPU partitioning helpers; it never computes parity itself.
"""
from ._lib import EXPORTED, LIB_PATH, Status, XecLibraryError, lib
from .codec import (DECODE_KERNELS, Pipeline, build_info, check_args, check_bitmap, decode,
                    decode_arg_capacity_used, decode_device, decode_device_list,
                    decode_per_stripe, decode_tiling_used,
                    device_list_bytes, encode, erase,
                    fill_splitmix64, init,
                    select_lost_blocks, set_decode_tiling, set_kernel_events, set_launch,
                    set_occupancy,
                    set_rotation, set_validate_kernel,
                    status_string, validate_blocks, write_validation_pattern)
from .partition import stripe_range

__all__ = [
    "DECODE_KERNELS", "EXPORTED", "LIB_PATH", "Pipeline", "Status", "XecLibraryError", "lib",
    "build_info", "check_args", "check_bitmap", "decode", "decode_arg_capacity_used",
    "decode_device", "decode_device_list",
    "decode_per_stripe", "decode_tiling_used", "device_list_bytes",
    "encode", "erase", "fill_splitmix64", "init", "select_lost_blocks", "set_decode_tiling",
    "set_kernel_events",
    "set_launch",
    "set_occupancy", "set_rotation", "set_validate_kernel", "status_string", "stripe_range", "validate_blocks",
    "write_validation_pattern",
]
