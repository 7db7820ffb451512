"""Multi-GPU plumbing for stripe-partitioned XOR-EC.

One process per GPU.  Stripes are independent, so the codec itself needs no
collective: each rank encodes / decodes the contiguous stripe range
:func:`xec.partition.stripe_range` assigns it.  The only exchanges are

* ``scatter_stripes`` -- the root hands each rank its slice of a batch that
  starts on the root (the reference's single-GPU batch, xorec_gpu_cmp_bm.cpp:
  25-37, spread over the node); point-to-point send/recv because ranges are
  ragged and RCCL has no scatter primitive; over xGMI with backend "nccl"
  (RCCL), over TCP with "gloo" (CPU tests);
* ``gather_stripes`` -- the inverse, e.g. parity or recovered blocks back to
  the root;
* ``max_over_ranks`` -- the timing reduction of bench.py.

The root's egress is bounded by its xGMI links, far below HBM bandwidth, so
scatter-inclusive rates are reported separately from the device-resident
metric.
"""
from __future__ import annotations

import os

from .partition import stripe_range

# Largest single point-to-point message.  RCCL 2.26 (torch 2.10's bundled
# librccl) returned a send-to-self of more than 1 GiB with its second half
# wrong and no error (tools/rccl/p2p_size_probe.py, profiles/r02bf), and
# config 5 sends 4 GiB per peer; every transfer is therefore posted as pieces
# of at most this many bytes, in offset order on both ends (matched pairwise
# in order).  XEC_P2P_PIECE_BYTES overrides it (tests).
P2P_PIECE_BYTES = 256 << 20


def _piece_bytes() -> int:
    return int(os.environ.get("XEC_P2P_PIECE_BYTES", P2P_PIECE_BYTES))


def _dist():
    import torch.distributed as dist
    return dist


def p2p_ops(op, tensor, peer):
    """P2POps moving the 1-D ``tensor`` to / from ``peer`` in pieces of at most
    :data:`P2P_PIECE_BYTES` bytes."""
    dist = _dist()
    step = max(1, _piece_bytes() // max(1, tensor.element_size()))
    n = tensor.numel()
    return [dist.P2POp(op, tensor[i:i + step], peer) for i in range(0, n, step)]


def _batch(ops):
    """Post `ops` as one batch and wait.  Both ends of every transfer go
    through batch_isend_irecv: with RCCL a batched op runs on the group's own
    communicator, while a plain send / recv would run on a separate two-rank
    communicator that the peer's batched op never joins."""
    dist = _dist()
    for w in (dist.batch_isend_irecv(ops) if ops else []):
        w.wait()


def scatter_stripes(full, local, S_total: int, stripe_bytes: int, root: int = 0):
    """Copy stripes [start, stop) of ``full`` (uint8, S_total*stripe_bytes, only
    read on ``root``) into ``local`` (uint8, (stop-start)*stripe_bytes) on every
    rank.  Returns ``local``."""
    dist = _dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    if rank == root:
        ops = []
        for r in range(world):
            a, b = stripe_range(S_total, r, world)
            piece = full[a * stripe_bytes:b * stripe_bytes]
            if r == root:
                local.copy_(piece)
            elif b > a:
                ops += p2p_ops(dist.isend, piece, r)
        _batch(ops)
    else:
        a, b = stripe_range(S_total, rank, world)
        if b > a:
            _batch(p2p_ops(dist.irecv, local, root))
    return local


def gather_stripes(local, full, S_total: int, stripe_bytes: int, root: int = 0):
    """Inverse of :func:`scatter_stripes`: every rank's ``local`` slice lands in
    ``full`` on ``root`` (``full`` is ignored elsewhere)."""
    dist = _dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    if rank == root:
        ops = []
        for r in range(world):
            a, b = stripe_range(S_total, r, world)
            piece = full[a * stripe_bytes:b * stripe_bytes]
            if r == root:
                piece.copy_(local)
            elif b > a:
                ops += p2p_ops(dist.irecv, piece, r)
        _batch(ops)
    else:
        a, b = stripe_range(S_total, rank, world)
        if b > a:
            _batch(p2p_ops(dist.isend, local, root))
    return full


def max_over_ranks(values, device=None):
    """Element-wise max of a list of floats over all ranks (bench timing)."""
    import torch
    dist = _dist()
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.tolist()
