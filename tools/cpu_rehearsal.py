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

    _events = None  # xec_set_kernel_events stand-in: (start, stop) for the next call

    def set_kernel_events(self, start, stop):
        self._events = (start, stop)
        return 0

    def _timed(self, fn):
        ev, self._events = self._events, None
        if ev and ev[0] is not None:
            ev[0].record()
        rc = fn()
        if ev and ev[1] is not None:
            ev[1].record()
        return rc

    def encode(self, d, p, S, bs, k, m, stream=None):
        return self._timed(lambda: self._encode(d, p, S, bs, k, m))

    def _encode(self, d, p, S, bs, k, m):
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
        return self._timed(lambda: self._rebuild(d, p, S, bs, k, m, _np(h_bm)))

    def decode_device(self, d, p, S, bs, k, m, d_bm, d_status, stream=None):
        _np(d_status)[0] = 0
        return self._timed(lambda: self._rebuild(d, p, S, bs, k, m, _np(d_bm)))

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


def multi_leg_main(argv):
    """Stand-in for erasure-code-benchmark_amd/bin/xec_multi_leg (bench.py's
    multi_device leg) with the same options and the same JSON keys, computed on
    the CPU: shards = the device list's stripe ranges, "scatter" = slice copies
    from a root batch, per-shard encode, "gather" = the parity slices back,
    compared with the root's own encode.  Measures nothing."""
    import argparse
    import json
    import sys
    ap = argparse.ArgumentParser(prog="cpu_rehearsal.py multi-leg")
    ap.add_argument("--devices", required=True)
    ap.add_argument("--stripes-per-device", type=int, default=256)
    ap.add_argument("--data", type=int, default=16)
    ap.add_argument("--parity", type=int, default=1)
    ap.add_argument("--block", type=int, default=1 << 20)
    a = ap.parse_args(argv)
    devices = [int(x) for x in a.devices.split(",")]
    k, m, bs, S_per = a.data, a.parity, a.block, a.stripes_per_device
    S = S_per * len(devices)
    # keep the rehearsal small whatever shape bench.py passes
    bs_r = min(bs, 4096)
    import torch
    x = CpuXec()
    root = torch.empty(S * k * bs_r, dtype=torch.uint8)
    x.fill_splitmix64(root, S, k * bs_r, 1896)
    ref = torch.empty(S * m * bs_r, dtype=torch.uint8)
    x.encode(root, ref, S, bs_r, k, m)
    t0 = time.perf_counter()
    gathered = torch.empty_like(ref)
    for i in range(len(devices)):
        a0, a1 = i * S_per, (i + 1) * S_per
        shard = root[a0 * k * bs_r:a1 * k * bs_r].clone()  # "scatter"
        par = torch.empty(S_per * m * bs_r, dtype=torch.uint8)
        x.encode(shard, par, S_per, bs_r, k, m)
        gathered[a0 * m * bs_r:a1 * m * bs_r] = par  # "gather"
    t = time.perf_counter() - t0
    exact = bool(torch.equal(gathered, ref))
    import os
    from xec import topology
    topo = (topology.record(devices[0], devices) if os.environ.get("XEC_TOPOLOGY_STUB")
            else {"skipped": "CPU rehearsal: no runtime to ask (set XEC_TOPOLOGY_STUB)"})
    out = {"plugin": "CPU REHEARSAL stand-in (tools/cpu_rehearsal.py): not a measurement",
           "rehearsal": True, "devices": devices, "k": k, "m": m, "block_bytes": bs,
           "stripes_per_device": S_per, "stripes_total": S,
           "distinct_devices": len(set(devices)), "encode_ms": round(t * 1e3, 4),
           "decode_ms": round(t * 1e3, 4), "value_GBps": 0.0, "bit_exact": exact,
           "topology": topo,
           "scatter": {"root": devices[0], "gathered_parity_bit_exact_vs_root_encode": exact,
                       "path": topo.get("path", "unknown")}}
    print(json.dumps(out))
    sys.exit(0 if exact else 1)


if __name__ == "__main__":
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "erasure-code-benchmark_amd"))
    if len(sys.argv) < 2 or sys.argv[1] != "multi-leg":
        sys.exit("usage: cpu_rehearsal.py multi-leg --devices LIST [...]")
    multi_leg_main(sys.argv[2:])
