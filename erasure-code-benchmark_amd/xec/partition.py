"""Stripe-batch partitioning across GPUs.

Stripes are independent (the reference parallelises over them with no
exchange, src/algorithms/xorec_bm.cpp:30), so a batch of S stripes is split
into contiguous ranges, one per rank; the first S % world ranks take one extra
stripe.  No collective is on the data path.
"""
from __future__ import annotations


def stripe_range(S: int, rank: int, world: int) -> tuple[int, int]:
    """[start, stop) of the stripes owned by ``rank`` out of ``world``."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(S, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


#: GPUs of one node in BASELINE.json configs[4] (config 5)
CONFIG5_GPUS = 8


def config5_devices(visible: int, gpus: int = CONFIG5_GPUS) -> list[int]:
    """The device list config 5's one-process tests run:
    the distinct devices 0 .. min(visible, gpus) - 1 whenever more than one GPU
    is visible, so the peer copies cross real links; on a one-GPU box device 0
    repeated `gpus` times, so the full shape still runs (its copies are device
    copies)."""
    if visible < 1:
        raise ValueError("no visible GPU")
    if visible >= 2:
        return list(range(min(visible, gpus)))
    return [0] * gpus
