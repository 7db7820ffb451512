#!/usr/bin/env python3
"""Does the physical placement of the parity buffer relative to the data
buffer change the encode rate?  (Probe for the in-place decode penalty,
DESIGN.md §3.)  One allocation; data at 0, parity at data_bytes + delta for a
set of deltas; interleaved rounds, HIP events.

    python tools/lab/offset_probe.py [--workload cfg3] [--rounds 5]
"""
from __future__ import annotations

import argparse
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))

from bench import algorithmic_bytes, workload_shape  # noqa: E402

DELTAS = [0, 4096, 65536, 1 << 20, (1 << 20) + 4096, (3 << 20) + 65536, 1 << 24, (1 << 27) + 4096]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import torch

    import xec

    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    k, m, bs, S, _ = workload_shape(args.workload)
    db, pb = S * k * bs, S * m * bs
    span = db + max(DELTAS) + pb
    bufs = [torch.empty(span, dtype=torch.uint8, device="cuda") for _ in range(2)]
    s = torch.cuda.current_stream()
    for i, b in enumerate(bufs):
        assert xec.fill_splitmix64(b[:db], S, k * bs, 1896 + i, s) == 0
    sep = [torch.empty(pb, dtype=torch.uint8, device="cuda") for _ in range(2)]
    b_enc, _ = algorithmic_bytes(S, k, m, bs)

    def run(parity_of):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.iters + 1)]
        xec.encode(bufs[0].data_ptr(), parity_of(0), S, bs, k, m, s)
        ev[0].record(s)
        for i in range(args.iters):
            xec.encode(bufs[i % 2].data_ptr(), parity_of(i % 2), S, bs, k, m, s)
            ev[i + 1].record(s)
        torch.cuda.synchronize()
        return [ev[i].elapsed_time(ev[i + 1]) for i in range(args.iters)]

    res = {f"delta_{d}": [] for d in DELTAS}
    res["separate_alloc"] = []
    for _ in range(args.rounds):
        for d in DELTAS:
            res[f"delta_{d}"] += run(lambda i, d=d: bufs[i].data_ptr() + db + d)
        res["separate_alloc"] += run(lambda i: sep[i].data_ptr())
    for n, ts in res.items():
        med = statistics.median(ts)
        print(f"{n:24s} enc_ms {med:.4f}  GBps {b_enc / med / 1e6:.1f}", flush=True)


if __name__ == "__main__":
    main()
