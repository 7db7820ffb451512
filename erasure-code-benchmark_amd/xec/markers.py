"""ROCTx ranges for profiling bench.py (rocprofv3), no effect otherwise.

bench.py pauses the profiler first thing and brackets its timed region with
:func:`timed_region`: ``roctxProfilerResume``, a ROCTx range named
``bench:timed``, ``roctxProfilerPause``.  Under
``rocprofv3 --marker-trace --kernel-trace --stats`` (tools/gpu_profile.sh) the
control calls are honoured, so the kernel trace and its stats hold exactly the
timed launches (ROCm 7.2, profiles/r03c: 5 of 11 probe launches traced; with
``--selected-regions`` instead, nothing at all was recorded).  The legs after
the headline (host pipeline, scatter) get ranges of their own.  Without a profiler attached
the calls are no-ops inside the ROCTx library.  This is measurement plumbing,
not the codec: when the ROCTx library is absent every function does nothing.
"""
from __future__ import annotations

import contextlib
import ctypes

_ROCTX = None
_LOADED = False
_NAMES = ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
          "librocprofiler-sdk-roctx.so")


def _roctx():
    global _ROCTX, _LOADED
    if _LOADED:
        return _ROCTX
    _LOADED = True
    for name in _NAMES:
        try:
            L = ctypes.CDLL(name)
        except OSError:
            continue
        L.roctxRangePushA.argtypes = [ctypes.c_char_p]
        L.roctxRangePushA.restype = ctypes.c_int
        L.roctxRangePop.argtypes = []
        L.roctxRangePop.restype = ctypes.c_int
        L.roctxProfilerPause.argtypes = [ctypes.c_uint64]
        L.roctxProfilerResume.argtypes = [ctypes.c_uint64]
        _ROCTX = L
        break
    return _ROCTX


def available() -> bool:
    return _roctx() is not None


@contextlib.contextmanager
def region(name: str):
    """A ROCTx range around the block (``--marker-trace`` shows it)."""
    L = _roctx()
    if L is not None:
        L.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if L is not None:
            L.roctxRangePop()


def pause() -> None:
    """roctxProfilerPause(0): under ``--selected-regions``, stop collecting."""
    L = _roctx()
    if L is not None:
        L.roctxProfilerPause(0)


def resume() -> None:
    """roctxProfilerResume(0): under ``--selected-regions``, collect from here."""
    L = _roctx()
    if L is not None:
        L.roctxProfilerResume(0)


@contextlib.contextmanager
def timed_region(name: str = "bench:timed"):
    """Collect (``--selected-regions``) and mark exactly the enclosed region."""
    resume()
    try:
        with region(name):
            yield
    finally:
        pause()
