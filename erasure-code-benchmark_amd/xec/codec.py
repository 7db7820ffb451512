"""Thin Python view of the C ABI (include/xec.h) for tests and bench.py.

Every function forwards to libxec_hip.so and returns the :class:`Status` the
library returned -- the same 0..4 codes as the reference XorecResult
(src/xorec/xorec_utils.hpp:26-32).  Device buffers are passed as integer
addresses or as torch tensors (``.data_ptr()``); streams as a
``torch.cuda.Stream``, a raw ``hipStream_t`` integer or ``None`` (null stream).
"""
from __future__ import annotations

import ctypes

from ._lib import Status, lib


def _ptr(x) -> int:
    if x is None:
        return 0
    if hasattr(x, "data_ptr"):
        return int(x.data_ptr())
    if hasattr(x, "ctypes"):  # numpy array (host memory)
        return int(x.ctypes.data)
    return int(x)


def _stream(s) -> int:
    if s is None:
        return 0
    if hasattr(s, "cuda_stream"):
        return int(s.cuda_stream)
    return int(s)


def init(device_id: int = 0) -> Status:
    """xec_init -- replaces xorec_gpu_init + xorec_init (xorec_gpu_cmp.cu:7-27)."""
    return Status(lib().xec_init(int(device_id)))


def encode(d_data, d_parity, S: int, bs: int, k: int, m: int, stream=None) -> Status:
    """xec_encode -- replaces xorec_gpu_encode (xorec_gpu_cmp.cu:29-55)."""
    return Status(lib().xec_encode(_ptr(d_data), _ptr(d_parity), S, bs, k, m, _stream(stream)))


def decode(d_data, d_parity, S: int, bs: int, k: int, m: int, h_bitmap, d_bitmap,
           stream=None) -> Status:
    """xec_decode -- replaces xorec_gpu_decode (xorec_gpu_cmp.cu:57-115); parity read-only."""
    return Status(lib().xec_decode(_ptr(d_data), _ptr(d_parity), S, bs, k, m, _ptr(h_bitmap),
                                   _ptr(d_bitmap), _stream(stream)))


def decode_per_stripe(d_data, d_parity, S: int, bs: int, k: int, m: int, h_bitmap, d_bitmap,
                      h_codes=None, stream=None) -> Status:
    """xec_decode_per_stripe -- the reference CPU plugin's per-stripe semantics
    (xorec_bm.cpp:43-58): recoverable stripes are rebuilt, unrecoverable ones
    left alone; h_codes (S host bytes, optional) gets each stripe's 0 / 4."""
    return Status(lib().xec_decode_per_stripe(_ptr(d_data), _ptr(d_parity), S, bs, k, m,
                                              _ptr(h_bitmap), _ptr(d_bitmap),
                                              _ptr(h_codes) if h_codes is not None else None,
                                              _stream(stream)))


def decode_device(d_data, d_parity, S: int, bs: int, k: int, m: int, d_bitmap, d_status,
                  stream=None) -> Status:
    """xec_decode_device -- bitmap already on the device; batch verdict lands in
    d_status (int32 device tensor: 0 or 4) in stream order, nothing is synchronised."""
    return Status(lib().xec_decode_device(_ptr(d_data), _ptr(d_parity), S, bs, k, m,
                                          _ptr(d_bitmap), _ptr(d_status), _stream(stream)))


def decode_device_list(d_data, d_parity, S: int, bs: int, k: int, m: int, d_bitmap, d_work,
                       work_bytes: int, d_status, stream=None) -> Status:
    """xec_decode_device_list -- as decode_device, but the check kernel lists the
    lost data blocks into d_work (device scratch of device_list_bytes(S, k, m)
    bytes) and only those are rebuilt: for batches where few stripes lost blocks."""
    return Status(lib().xec_decode_device_list(_ptr(d_data), _ptr(d_parity), S, bs, k, m,
                                               _ptr(d_bitmap), _ptr(d_work), work_bytes,
                                               _ptr(d_status), _stream(stream)))


def device_list_bytes(S: int, k: int, m: int) -> int:
    """xec_decode_device_list_bytes: scratch decode_device_list needs."""
    return int(lib().xec_decode_device_list_bytes(S, k, m))


def erase(d_data, d_parity, S: int, bs: int, k: int, m: int, d_bitmap, stream=None) -> Status:
    """xec_erase -- device-side simulate_data_loss (abstract_bm.cpp:20-39)."""
    return Status(lib().xec_erase(_ptr(d_data), _ptr(d_parity), S, bs, k, m, _ptr(d_bitmap),
                                  _stream(stream)))


def fill_splitmix64(d_buf, S: int, stripe_bytes: int, seed_base: int, stream=None) -> Status:
    return Status(lib().xec_fill_splitmix64(_ptr(d_buf), S, stripe_bytes, seed_base,
                                            _stream(stream)))


def write_validation_pattern(d_data, nblocks: int, bs: int, seed: int, stream=None) -> Status:
    """xec_write_validation_pattern -- utils.cpp:35-69 on the device."""
    return Status(lib().xec_write_validation_pattern(_ptr(d_data), nblocks, bs, seed,
                                                     _stream(stream)))


def validate_blocks(d_data, nblocks: int, bs: int, d_bad, stream=None) -> Status:
    """xec_validate_blocks -- utils.cpp:72-97 on the device; *d_bad = failing blocks."""
    return Status(lib().xec_validate_blocks(_ptr(d_data), nblocks, bs, _ptr(d_bad),
                                            _stream(stream)))


def check_bitmap(h_bitmap, S: int, k: int, m: int) -> tuple[Status, bool]:
    """Host-only recoverability scan; returns (status, needs_recovery)."""
    needs = ctypes.c_int(0)
    st = Status(lib().xec_check_bitmap(_ptr(h_bitmap), S, k, m, ctypes.byref(needs)))
    return st, bool(needs.value)


def select_lost_blocks(k: int, m: int, lost: int, h_bitmap, seed: int) -> Status:
    """xec_select_lost_blocks -- utils.cpp:100-127 with an explicit seed, on one
    stripe's (k+m)-byte host bitmap (host only)."""
    return Status(lib().xec_select_lost_blocks(k, m, lost, _ptr(h_bitmap), seed))


def check_args(data_addr: int, parity_addr: int, bs: int, k: int, m: int) -> Status:
    """Host-only xorec_check_args (xorec_utils.hpp:61-86)."""
    return Status(lib().xec_check_args(data_addr, parity_addr, bs, k, m))


def set_launch(unroll: int = 0, max_grid: int = 0, cache_policy: int = 0,
               block_threads: int = 0) -> Status:
    """xec_set_launch; 0 = default for each; cache_policy 1 = nt, 2 = default policy;
    block_threads 64 or 256."""
    return Status(lib().xec_set_launch(unroll, max_grid, cache_policy, block_threads))


def set_occupancy(waves_per_simd: int = 0) -> Status:
    """xec_set_occupancy; resident encode/decode waves per SIMD (1..8, 8 = no cap),
    0 = automatic (measured per member count; the default)."""
    return Status(lib().xec_set_occupancy(waves_per_simd))


def set_decode_tiling(tiling: int = 0) -> Status:
    """xec_set_decode_tiling; 0 = automatic (default), 1 = stripe tiles, 2 = class tiles
    (m > 1 only), 3 = work-list tiles where the list fits, 4 = kernel-argument mask
    tiles where they apply (S <= 1,024, k <= 32) (identical results)."""
    return Status(lib().xec_set_decode_tiling(tiling))


def set_rotation(tiles: int = 0) -> Status:
    """xec_set_rotation: column rotation of the tile kernels (this thread)."""
    return Status(lib().xec_set_rotation(tiles))


def set_validate_kernel(mode: int = 0) -> Status:
    """xec_set_validate_kernel; 0 = automatic (default), 1 = lane per block,
    2 = wave per block (identical results)."""
    return Status(lib().xec_set_validate_kernel(mode))


#: xec_decode_tiling_used values (include/xec.h)
DECODE_KERNELS = {1: "xec::decode_kernel", 2: "xec::decode_class_kernel",
                  3: "xec::decode_list_kernel", 4: "xec::decode_arglist_kernel",
                  5: "xec::decode_argmask_kernel", 6: "xec::decode_argmask_kernel"}


def decode_tiling_used() -> int:
    """xec_decode_tiling_used: the tiling this thread's last xec_decode launched
    (0 none, 1 stripe, 2 class, 3 device list, 4 kernel-argument list,
    5 kernel-argument masks over class tiles, 6 the same over stripe tiles)."""
    return int(lib().xec_decode_tiling_used())


def set_kernel_events(start, stop) -> Status:
    """xec_set_kernel_events: the calling thread's next codec call launches its
    kernel with these events, recorded by the kernel's own dispatch
    (hipExtLaunchKernel); `start` / `stop` are torch.cuda.Event objects (or
    None).  torch creates an event's HIP handle at its first record(), so each
    must have been recorded once before."""
    def handle(ev):
        if ev is None:
            return None
        h = int(ev.cuda_event)
        if not h:
            raise ValueError("record the torch.cuda.Event once before handing it over")
        return ctypes.c_void_p(h)
    return Status(lib().xec_set_kernel_events(handle(start), handle(stop)))


def decode_arg_capacity_used() -> int:
    """xec_decode_arg_capacity_used: after a kernel-argument list decode, the
    capacity its arguments carried (64, 256 or 1024 entries); else 0."""
    return int(lib().xec_decode_arg_capacity_used())


def status_string(st: int) -> str:
    return lib().xec_status_string(int(st)).decode()


def build_info() -> str:
    return lib().xec_build_info().decode()


class Pipeline:
    """Host-in / host-out encoder-decoder (xec_pipeline_*, include/xec.h).

    Owns ``nstreams`` device slots of ``chunk_stripes`` stripes on the current
    device; host buffers (numpy arrays, pinned torch tensors or addresses) are
    streamed through them.  Use as a context manager or call :meth:`close`."""

    def __init__(self, chunk_stripes: int, bs: int, k: int, m: int, nstreams: int = 2):
        self.bs, self.k, self.m = bs, k, m
        h = ctypes.c_void_p()
        st = Status(lib().xec_pipeline_create(ctypes.byref(h), chunk_stripes, bs, k, m, nstreams))
        if st != Status.SUCCESS:
            raise RuntimeError(f"xec_pipeline_create failed: {st!r}")
        self._h = h

    def encode(self, h_data, h_parity, S: int) -> Status:
        return Status(lib().xec_pipeline_encode(self._h, _ptr(h_data), _ptr(h_parity), S))

    def decode(self, h_data, h_parity, S: int, h_bitmap) -> Status:
        return Status(lib().xec_pipeline_decode(self._h, _ptr(h_data), _ptr(h_parity), S,
                                                _ptr(h_bitmap)))

    def close(self) -> None:
        if self._h:
            lib().xec_pipeline_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter teardown
            pass
