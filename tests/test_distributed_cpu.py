"""N>1 path on CPU: gloo, world_size 2, 3, 4 and 8, ragged stripe partitions (empty ranks at S < world).

Each rank encodes its own stripe range (oracle encode stands in for the GPU
kernel: the point here is the partition / scatter / gather / timing logic
that bench.py uses at N>1), the root gathers parity, and the result must equal
the single-process encode of the whole batch bit for bit.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import xorec_oracle as xo
from xec.partition import stripe_range


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, S, k, m, bs, out_q):
    import torch.distributed as dist

    from xec import dist as xdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o = xo.COracle()
        stripe = k * bs
        full = None
        if rank == 0:
            d, _ = o.batch(S, k, m, bs)
            full = torch.from_numpy(d.copy())
        a, b = stripe_range(S, rank, world)
        local = torch.empty((b - a) * stripe, dtype=torch.uint8)
        xdist.scatter_stripes(full, local, S, stripe)
        # every rank must hold exactly its slice of the root's batch
        want = xo.make_data(S, k, bs).reshape(-1)[a * stripe:b * stripe]
        assert np.array_equal(local.numpy(), want)
        ld = xo.COracle.aligned(local.numel())
        ld[:] = local.numpy()
        lp = xo.COracle.aligned((b - a) * m * bs)
        assert o.encode_batch(ld, lp, b - a, bs, k, m, 1) == 0
        par_full = torch.empty(S * m * bs, dtype=torch.uint8) if rank == 0 else None
        xdist.gather_stripes(torch.from_numpy(lp.copy()), par_full, S, m * bs)
        t = xdist.max_over_ranks([float(rank + 1), -float(rank)])
        assert t == [float(world), 0.0]
        if rank == 0:
            out_q.put(par_full.numpy().tobytes())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,S,piece", [(2, 9, 0), (2, 2, 0), (3, 10, 0), (3, 2, 0), (4, 9, 0),
                                           (8, 20, 0), (8, 5, 0),
                                           # transfers split into ragged pieces (xec/dist.py
                                           # P2P_PIECE_BYTES): 1000 B against 4 KiB stripes
                                           (3, 10, 1000), (4, 9, 4096)])
def test_partitioned_encode_matches_single_process(world, S, piece, monkeypatch):
    k, m, bs = 8, 2, 512
    if piece:  # inherited by the spawned ranks
        monkeypatch.setenv("XEC_P2P_PIECE_BYTES", str(piece))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, S, k, m, bs, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    o = xo.COracle()
    _, ref_p = o.batch(S, k, m, bs)
    assert got == ref_p.tobytes()


def test_stripe_range_properties():
    for S in range(0, 40):
        for world in range(1, 9):
            ranges = [stripe_range(S, r, world) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == S
            for (a0, b0), (a1, _) in zip(ranges, ranges[1:]):
                assert b0 == a1
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        stripe_range(4, 2, 2)


class _CpuOps:
    """CPU stand-ins for bench.DeviceOps: the oracle's fill and encode (test
    infrastructure), so bench.measure_scatter's scatter -> encode -> gather ->
    verify logic runs under gloo exactly as it does over RCCL."""
    device = "cpu"

    def __init__(self, k, m, bs):
        self.o, self.k, self.m, self.bs = xo.COracle(), k, m, bs

    def fill(self, buf, S, seed_base):
        if S:
            d, _ = self.o.batch(S, self.k, self.m, self.bs, seed_base=seed_base)
            buf.copy_(torch.from_numpy(d.reshape(-1).copy()))

    def encode(self, d, p, S):
        if S:
            ld = xo.COracle.aligned(d.numel())
            ld[:] = d.numpy()
            lp = xo.COracle.aligned(S * self.m * self.bs)
            assert self.o.encode_batch(ld, lp, S, self.bs, self.k, self.m, 1) == 0
            p.copy_(torch.from_numpy(lp.copy()))

    def sync(self):
        pass


def _bench_worker(rank, world, port, S_total, k, m, bs, out_q):
    import torch.distributed as dist

    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, b = stripe_range(S_total, rank, world)
        r = bench.measure_scatter(torch, dist, _CpuOps(k, m, bs), S_total, b - a, a, k, m, bs,
                                  enc_ms=1.0, reps=1)
        if rank == 0:
            out_q.put(r)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,S", [(2, 7), (3, 10), (3, 2)])
def test_bench_scatter_gather_leg(world, S):
    """bench.py's N>1 RCCL leg (scatter, per-rank encode, parity gather, checks
    against the root's own whole-batch encode), run under gloo on the CPU."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, S, 8, 2, 512, q))
             for r in range(world)]
    for p in procs:
        p.start()
    r = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert r["bit_exact"] is True
    assert r["gathered_parity_bit_exact_vs_root_encode"] is True
    assert r["scatter_ms"] > 0 and r["gather_parity_ms"] > 0
