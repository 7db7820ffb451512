#!/usr/bin/env python3
"""Does bench.py's per-kernel timing cost the step anything?  (lab, not the product)

bench.py records three HIP events per timed step (before encode, between
encode and decode, after decode) to report each kernel's average duration.
This times the same steps -- config 3, three resident sets in rotation, the
C ABI on torch's current stream, exactly bench.py's step -- with and without
those events, interleaved over several rounds in one process, and reports
ms per step for each mode: "none"; "events" (bench.py's three per step);
"chain" (one event between every two kernels: step i's decode-end event is
step i+1's encode-start); "ends" (two events around the whole loop only).

    python tools/lab/event_cost.py [--steps 50] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch
    import xec
    import bench

    k, m, bs, S, _ = bench.workload_shape("cfg3")
    assert xec.init(0) == 0
    stream = torch.cuda.current_stream()
    sets = []
    for s in range(bench.NSETS):
        d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
        p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
        assert xec.fill_splitmix64(d, S, k * bs, bench.SEED + s * (1 << 40), stream) == 0
        assert xec.encode(d, p, S, bs, k, m, stream) == 0
        sets.append((d, p))
    h_bm = torch.from_numpy(bench.erasure_pattern(np, S, k, m).reshape(-1)).pin_memory()
    scratch = [torch.empty(h_bm.numel(), dtype=torch.uint8, device="cuda")
               for _ in range(bench.NSETS)]

    def step(i, ev=None):
        de, pe = sets[i % bench.NSETS]
        di = (i + bench.NSETS - 1) % bench.NSETS
        dd, pd = sets[di]
        if ev is not None:
            ev[0].record(stream)
        rc = xec.encode(de, pe, S, bs, k, m, stream)
        if ev is not None:
            ev[1].record(stream)
        rc |= xec.decode(dd, pd, S, bs, k, m, h_bm, scratch[di], stream)
        if ev is not None:
            ev[2].record(stream)
        return rc

    for i in range(10):
        assert step(i) == 0
    torch.cuda.synchronize()

    def chain_step(i, ev):
        de, pe = sets[i % bench.NSETS]
        di = (i + bench.NSETS - 1) % bench.NSETS
        dd, pd = sets[di]
        rc = xec.encode(de, pe, S, bs, k, m, stream)
        ev[2 * i + 1].record(stream)
        rc |= xec.decode(dd, pd, S, bs, k, m, h_bm, scratch[di], stream)
        ev[2 * i + 2].record(stream)
        return rc

    res = {"none": [], "events": [], "chain": [], "ends": []}
    for r in range(args.rounds):
        for mode in ("none", "events", "chain", "ends"):
            evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)]
                   for _ in range(args.steps)] if mode == "events" else None
            ch = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.steps + 1)] \
                if mode == "chain" else None
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if mode == "ends":
                e0.record(stream)
            if mode == "chain":
                ch[0].record(stream)
            rc = 0
            for i in range(args.steps):
                rc |= chain_step(i, ch) if ch else step(i, evs[i] if evs else None)
            if mode == "ends":
                e1.record(stream)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps * 1e3
            assert rc == 0
            row = {"round": r, "wall_ms_per_step": round(dt, 4)}
            if mode == "ends":
                row["event_ms_per_step"] = round(e0.elapsed_time(e1) / args.steps, 4)
            if mode == "chain":
                row["enc_ms"] = round(sum(ch[2 * i].elapsed_time(ch[2 * i + 1])
                                          for i in range(args.steps)) / args.steps, 4)
                row["dec_ms"] = round(sum(ch[2 * i + 1].elapsed_time(ch[2 * i + 2])
                                          for i in range(args.steps)) / args.steps, 4)
            if mode == "events":
                row["enc_ms"] = round(sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps, 4)
                row["dec_ms"] = round(sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps, 4)
            res[mode].append(row)
            print(mode, json.dumps(row), flush=True)
    summary = {m: round(sorted(x["wall_ms_per_step"] for x in v)[len(v) // 2], 4)
               for m, v in res.items()}
    print(json.dumps({"median_wall_ms_per_step": summary, "steps": args.steps,
                      "rounds": args.rounds}))


if __name__ == "__main__":
    main()
