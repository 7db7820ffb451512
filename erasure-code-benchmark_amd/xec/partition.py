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
