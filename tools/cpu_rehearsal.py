"""CPU stand-ins for bench.py's device calls -- `bench.py --rehearse-cpu` ONLY.

This exists so the N>1 launcher, the rank bookkeeping, the gloo collectives and
the JSON line of bench.py can be exercised on a machine without a GPU
(tests/test_bench_launcher.py).  It is never selected automatically: without
`--rehearse-cpu` bench.py loads libxec_hip.so or fails.  A rehearsal line says
so in its "data" field and its numbers are not measurements.

The stand-ins mirror the shape of the ``xec`` package calls bench.py makes
(same argument order, Status-like int returns) and of the few ``torch.cuda``
calls it makes (synchronize, Event, current_stream, set_device).
"""
from __future__ import annotations

import time

import numpy as np

_M = np.uint64


def _splitmix(seed: int, n: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = _M(seed) + np.arange(1, n + 1, dtype=np.uint64) * _M(0x9E3779B97F4A7C15)
        z = (z ^ (z >> _M(30))) * _M(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> _M(27))) * _M(0x94D049BB133111EB)
        return z ^ (z >> _M(31))


def _np(t):
    return t.numpy()


class CpuXec:
    """The subset of ``xec`` bench.py uses, on CPU torch tensors."""

    class Status(int):
        SUCCESS = 0

    def init(self, dev):
        return 0

    def stripe_range(self, S, rank, world):
        from xec.partition import stripe_range
        return stripe_range(S, rank, world)

    def fill_splitmix64(self, buf, S, stripe_bytes, seed_base, stream=None):
        v = _np(buf)[: S * stripe_bytes].view(np.uint64).reshape(S, stripe_bytes // 8)
        for c in range(S):
            v[c] = _splitmix(seed_base + c, stripe_bytes // 8)
        return 0

    def encode(self, d, p, S, bs, k, m, stream=None):
        if S == 0:
            return 0
        blocks = _np(d)[: S * k * bs].reshape(S, k // m, m, bs)
        _np(p)[: S * m * bs].reshape(S, m, bs)[:] = np.bitwise_xor.reduce(blocks, axis=1)
        return 0

    def _rebuild(self, d, p, S, bs, k, m, bm):
        data = _np(d)[: S * k * bs].reshape(S, k, bs)
        par = _np(p)[: S * m * bs].reshape(S, m, bs)
        rows = np.asarray(bm).reshape(S, k + m)
        for c, i in zip(*np.nonzero(rows[:, :k] == 0)):
            j = i % m
            others = [x for x in range(j, k, m) if x != i]
            data[c, i] = np.bitwise_xor.reduce(np.concatenate([par[c, j:j + 1], data[c, others]]),
                                               axis=0)
        return 0

    def decode(self, d, p, S, bs, k, m, h_bm, d_bm=None, stream=None):
        return self._rebuild(d, p, S, bs, k, m, _np(h_bm))

    def decode_device(self, d, p, S, bs, k, m, d_bm, d_status, stream=None):
        _np(d_status)[0] = 0
        return self._rebuild(d, p, S, bs, k, m, _np(d_bm))

    def erase(self, d, p, S, bs, k, m, d_bm, stream=None):
        data = _np(d)[: S * k * bs].reshape(S, k, bs)
        rows = _np(d_bm).reshape(S, k + m)
        for c, i in zip(*np.nonzero(rows[:, :k] == 0)):
            data[c, i] = 0
        return 0


class _Event:
    def __init__(self, enable_timing=True):
        self.t = 0.0

    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class CpuCuda:
    """The subset of ``torch.cuda`` bench.py uses."""
    Event = _Event

    def device_count(self):
        return 1

    def set_device(self, dev):
        pass

    def synchronize(self):
        pass

    def current_stream(self):
        return None
