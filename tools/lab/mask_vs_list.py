#!/usr/bin/env python3
"""Kernel-argument masks against the kernel-argument list at the reference's
8 MiB rows with losses (rows 1123-1126: (40/32), 1 KiB blocks, 256 stripes,
1 / 2 / 4 / 8 blocks drawn per stripe by the reference's select_lost_blocks).

The automatic policy sends a list of up to 1,024 lost blocks in the kernel
arguments (rows 1123-1125) and loss masks past that (row 1126).
This times one synchronous decode call (decode + stream synchronise, wall
clock) and the decode kernel from its own dispatch under the automatic choice
(0) and forced masks (4), alternating in one process; every variant's rebuilt
data is checked against the pristine batch.

    python tools/lab/mask_vs_list.py [--rounds 5] [--iters 400] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import numpy as np
    import torch

    import xec
    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for e in ev:
        e.record(s)
    k, m, bs, S = 32, 8, 1024, 256
    d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
    p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
    assert xec.fill_splitmix64(d, S, k * bs, 1896, s) == 0
    assert xec.encode(d, p, S, bs, k, m, s) == 0
    pristine = d.clone()
    out = []
    for lost in (1, 2, 4, 8):
        bm = np.ones((S, k + m), np.uint8)
        for c in range(S):
            assert xec.select_lost_blocks(k, m, lost, bm[c], 1000 * lost + c) == 0
        h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
        d_bm = h_bm.to("cuda")
        scratch = torch.empty_like(d_bm)
        used = {}
        for t in (0, 4):
            assert xec.set_decode_tiling(t) == 0
            d.copy_(pristine)  # the erase zeroes lost parity too: re-encode it each time
            assert xec.encode(d, p, S, bs, k, m, s) == 0
            assert xec.erase(d, p, S, bs, k, m, d_bm, s) == 0
            assert xec.decode(d, p, S, bs, k, m, h_bm, scratch, s) == 0
            torch.cuda.synchronize()
            used[t] = xec.decode_tiling_used()
            assert torch.equal(d, pristine), (lost, t)
        times = {t: {"call": [], "kernel": []} for t in (0, 4)}
        for _ in range(args.rounds):
            for t in (0, 4):
                assert xec.set_decode_tiling(t) == 0
                for i in range(args.iters + 20):
                    xec.set_kernel_events(ev[0], ev[1])
                    t0 = time.perf_counter()
                    assert xec.decode(d, p, S, bs, k, m, h_bm, scratch, s) == 0
                    s.synchronize()
                    t1 = time.perf_counter()
                    if i >= 20:
                        times[t]["call"].append((t1 - t0) * 1e6)
                        times[t]["kernel"].append(ev[0].elapsed_time(ev[1]) * 1e3)
        xec.set_decode_tiling(0)
        row = {"lost_per_stripe": lost, "lost_data": int((bm[:, :k] == 0).sum())}
        for t in (0, 4):
            row[f"tiling{t}"] = {"used": used[t],
                                 "call_us": round(statistics.median(times[t]["call"]), 2),
                                 "kernel_us": round(statistics.median(times[t]["kernel"]), 2)}
        print(json.dumps(row), flush=True)
        out.append(row)
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
