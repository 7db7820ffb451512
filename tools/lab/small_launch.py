#!/usr/bin/env python3
"""Launch shapes at the reference's 8 MiB messages (DESIGN.md §4 *Small messages*).

At 8 MiB a whole batch is 1,024-4,096 one-wave workgroups, one generation of
waves: the encode kernel takes ~4.3 us from its dispatch for what HBM moves in
~1.5 us.  Residency caps 1-8 changed nothing (profiles/r06e).  This times the
other launch knobs the library already has (xec_set_launch: block_threads 64
or 256, unroll 1 or 2 granules per lane; no rebuild) on the shapes of the
reference's 24 rows at 8 MiB (tools/reference_gpu_rows.csv), in one process,
variants interleaved round by round:

  kernel_us   the encode / decode kernel from its own dispatch
              (xec_set_kernel_events, hipExtLaunchKernel)
  call_us     encode() or decode() + stream synchronise, wall clock (Python
              adds the same few us to every variant)

Every variant's parity and rebuilt data are compared with the default's.

    python tools/lab/small_launch.py [--rounds 5] [--iters 40] [--out f.json]
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

MESSAGE = 8 << 20
# (k, m) of the reference's EC labels "(n/k)" at 8 MiB
ECS = [(8, 4), (16, 4), (16, 8), (32, 4), (32, 8)]
BLOCKS = [1024, 2048, 4096, 8192]


def variants_for(bs):
    v = [("default", 0, 0), ("u2", 2, 0)]
    if bs >= 4096:
        v += [("t256", 0, 256), ("t256u2", 2, 256)] if bs >= 8192 else [("t256", 0, 256)]
    return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=40)
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
    torch.cuda.synchronize()
    rows = []
    for bs in BLOCKS:
        for k, m in ECS:
            S = MESSAGE // (k * bs)
            d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
            p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
            assert xec.fill_splitmix64(d, S, k * bs, 1896, s) == 0
            bm = np.ones((S, k + m), np.uint8)
            bm[np.arange(S), (7 * np.arange(S)) % k] = 0  # one lost data block per stripe
            h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
            d_bm = torch.empty(S * (k + m), dtype=torch.uint8, device="cuda")
            variants = variants_for(bs)

            def run(op, unroll, threads):
                assert xec.set_launch(unroll, 0, 0, threads) == 0
                try:
                    if op == "encode":
                        return xec.encode(d, p, S, bs, k, m, s)
                    return xec.decode(d, p, S, bs, k, m, h_bm, d_bm, s)
                finally:
                    xec.set_launch(0, 0, 0, 0)

            ref_p = ref_d = None
            for name, u, t in variants:  # identical bytes from every variant
                p.zero_()
                assert run("encode", u, t) == 0
                torch.cuda.synchronize()
                ref_p = p.clone() if ref_p is None else ref_p
                assert torch.equal(p, ref_p), (bs, k, m, name)
                golden = d.clone()
                assert xec.erase(d, p, S, bs, k, m, d_bm.copy_(h_bm), s) == 0
                assert run("decode", u, t) == 0
                torch.cuda.synchronize()
                assert torch.equal(d, golden), (bs, k, m, name, "decode")
                ref_d = golden
            del ref_p, ref_d
            res = {(n, op): {"kernel": [], "call": []} for n, _, _ in variants
                   for op in ("encode", "decode")}
            for _ in range(args.rounds):
                for name, u, t in variants:
                    for op in ("encode", "decode"):
                        r = res[(name, op)]
                        for i in range(args.iters + 3):
                            xec.set_kernel_events(ev[0], ev[1])
                            t0 = time.perf_counter()
                            assert run(op, u, t) == 0
                            s.synchronize()
                            t1 = time.perf_counter()
                            if i >= 3:
                                r["call"].append((t1 - t0) * 1e6)
                                r["kernel"].append(ev[0].elapsed_time(ev[1]) * 1e3)
            row = {"bs": bs, "k": k, "m": m, "S": S, "tiles_1KiB": S * m * bs // 1024}
            for (name, op), r in res.items():
                row[f"{op}_{name}"] = {"kernel_us": round(statistics.median(r["kernel"]), 3),
                                       "call_us": round(statistics.median(r["call"]), 3)}
            print(json.dumps(row), flush=True)
            rows.append(row)
            del d, p, d_bm
    if args.out:
        Path(args.out).write_text(json.dumps(rows, indent=1) + "\n")


if __name__ == "__main__":
    main()
