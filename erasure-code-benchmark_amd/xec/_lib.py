"""ctypes binding of libxec_hip.so (the C ABI in include/xec.h).

The library is the product: there is no Python or CPU fallback.  A missing or
unloadable library raises :class:`XecLibraryError` immediately.

PyTorch ships its own HIP runtime (torch/lib/libamdhip64.so, SONAME
libamdhip64.so.7).  When torch is importable it is imported *before* the
library is loaded so that the dynamic loader resolves libxec_hip.so's
libamdhip64.so.7 dependency to that already-loaded copy: one HIP runtime per
process, so torch's device pointers and streams are valid in xec calls.
"""
from __future__ import annotations

import ctypes
import enum
import os
from pathlib import Path

LIB_NAME = "libxec_hip.so"
LIB_PATH = Path(os.environ.get("XEC_LIB", Path(__file__).resolve().parent / LIB_NAME))

#: every symbol include/xec.h declares (checked by tests/test_abi.py)
EXPORTED = (
    "xec_init", "xec_encode", "xec_decode", "xec_check_bitmap", "xec_check_args",
    "xec_erase", "xec_fill_splitmix64", "xec_set_launch", "xec_status_string",
    "xec_build_info", "xec_pipeline_create", "xec_pipeline_destroy", "xec_pipeline_encode",
    "xec_pipeline_decode", "xec_write_validation_pattern", "xec_validate_blocks",
    "xec_decode_device", "xec_set_occupancy", "xec_set_decode_tiling",
    "xec_set_validate_kernel", "xec_decode_tiling_used", "xec_decode_per_stripe",
    "xec_decode_device_list", "xec_decode_device_list_bytes", "xec_get_tuning",
    "xec_set_tuning", "xec_set_rotation", "xec_select_lost_blocks",
    "xec_decode_arg_capacity_used", "xec_peer_link", "xec_set_kernel_events",
)


class Tuning(ctypes.Structure):
    """xec_tuning (include/xec.h): the calling thread's overrides."""
    _fields_ = [(n, ctypes.c_int) for n in ("unroll", "max_grid", "cache_policy",
                                            "block_threads", "waves_per_simd",
                                            "decode_tiling", "validate_kernel", "rotation")]


class XecLibraryError(RuntimeError):
    pass


class Status(enum.IntEnum):
    """xec_status; 0..4 == reference XorecResult (xorec_utils.hpp:26-32)."""
    SUCCESS = 0
    INVALID_SIZE = 1
    INVALID_ALIGNMENT = 2
    INVALID_COUNTS = 3
    DECODE_FAILURE = 4
    NOT_INITIALIZED = 5
    DEVICE_ERROR = 6


_lib = None


def _share_torch_runtime() -> None:
    try:  # noqa: SIM105 -- torch is plumbing only; absent is fine on CPU-only hosts
        import torch  # noqa: F401
    except ImportError:
        pass


def lib() -> ctypes.CDLL:
    """Load (once) and return libxec_hip.so with argtypes set."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise XecLibraryError(
            f"{LIB_PATH} not found: build it with `make -C erasure-code-benchmark_amd` "
            "or __graft_entry__.build(); there is no fallback path")
    _share_torch_runtime()
    try:
        L = ctypes.CDLL(str(LIB_PATH))
    except OSError as e:  # pragma: no cover - depends on host
        raise XecLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    sz, vp, st = ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int
    sig = {
        "xec_init": ([ctypes.c_int], st),
        "xec_encode": ([vp, vp, sz, sz, sz, sz, vp], st),
        "xec_decode": ([vp, vp, sz, sz, sz, sz, vp, vp, vp], st),
        "xec_check_bitmap": ([vp, sz, sz, sz, ctypes.POINTER(ctypes.c_int)], st),
        "xec_check_args": ([vp, vp, sz, sz, sz], st),
        "xec_erase": ([vp, vp, sz, sz, sz, sz, vp, vp], st),
        "xec_fill_splitmix64": ([vp, sz, sz, ctypes.c_uint64, vp], st),
        "xec_set_launch": ([ctypes.c_int] * 4, st),
        "xec_set_occupancy": ([ctypes.c_int], st),
        "xec_set_decode_tiling": ([ctypes.c_int], st),
        "xec_set_validate_kernel": ([ctypes.c_int], st),
        "xec_decode_tiling_used": ([], ctypes.c_int),
        "xec_decode_arg_capacity_used": ([], ctypes.c_int),
        "xec_peer_link": ([ctypes.c_int, ctypes.c_int, vp], st),
        "xec_set_kernel_events": ([vp, vp], st),
        "xec_decode_per_stripe": ([vp, vp, sz, sz, sz, sz, vp, vp, vp, vp], st),
        "xec_status_string": ([st], ctypes.c_char_p),
        "xec_build_info": ([], ctypes.c_char_p),
        "xec_pipeline_create": ([ctypes.POINTER(vp), sz, sz, sz, sz, ctypes.c_int], st),
        "xec_pipeline_destroy": ([vp], st),
        "xec_pipeline_encode": ([vp, vp, vp, sz], st),
        "xec_pipeline_decode": ([vp, vp, vp, sz, vp], st),
        "xec_write_validation_pattern": ([vp, sz, sz, ctypes.c_uint64, vp], st),
        "xec_validate_blocks": ([vp, sz, sz, vp, vp], st),
        "xec_decode_device": ([vp, vp, sz, sz, sz, sz, vp, vp, vp], st),
        "xec_decode_device_list": ([vp, vp, sz, sz, sz, sz, vp, vp, sz, vp, vp], st),
        "xec_decode_device_list_bytes": ([sz, sz, sz], sz),
        "xec_set_rotation": ([ctypes.c_int], st),
        "xec_get_tuning": ([ctypes.POINTER(Tuning)], st),
        "xec_set_tuning": ([ctypes.POINTER(Tuning)], st),
        "xec_select_lost_blocks": ([sz, sz, sz, vp, ctypes.c_uint64], st),
    }
    default = "XEC_LIB" not in os.environ
    for name, (args, res) in sig.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            if default:
                raise XecLibraryError(f"{LIB_PATH} lacks {name}: rebuild it") from None
            continue  # an older build under XEC_LIB (in-process A/B, tools/ab): bind what it has
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L
