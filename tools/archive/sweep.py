#!/usr/bin/env python3
"""Launch-shape sweep for the XOR-EC kernels on one MI355X (one process,
interleaved rounds, HIP-event timing on the launching stream).

Also times two known-good HBM references on the same device and buffers size:
torch's device-to-device copy (copy_) and a torch.bitwise_xor of two tensors,
so kernel fractions can be read against what this box actually sustains.

    python tools/archive/sweep.py [--workload cfg3] [--rounds 5] [--iters 10]
"""
from __future__ import annotations

import argparse
import itertools
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))
sys.path.insert(0, str(ROOT))

from bench import WORKLOADS, algorithmic_bytes, erasure_pattern  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3",
                    help="bench.py workload name, or k,m,bs,S (e.g. 16,4,65536,4096)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--unroll", default="1,2")
    ap.add_argument("--threads", default="64,256")
    ap.add_argument("--grid", default="0,2048,4096")
    ap.add_argument("--nt", default="1,2", help="cache policy: 1 nt, 2 default")
    ap.add_argument("--occ", default="0", help="waves-per-SIMD caps (xec_set_occupancy): 0 = automatic, 8 = none")
    ap.add_argument("--lost", type=int, default=1,
                    help="lost data blocks per stripe (<= m, one per parity class)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import numpy as np
    import torch

    import xec

    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    if args.workload in WORKLOADS:
        k, m, bs, S, _ = WORKLOADS[args.workload]
    else:
        k, m, bs, S = (int(x) for x in args.workload.split(","))
    s = torch.cuda.current_stream()
    sets = []
    for i in range(2):
        d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
        p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
        assert xec.fill_splitmix64(d, S, k * bs, 1896 + i * 100000, s) == 0
        assert xec.encode(d, p, S, bs, k, m, s) == 0
        sets.append((d, p))
    bm = erasure_pattern(np, S, k, m, args.lost)  # bench.py: one per class per stripe
    h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
    scratch = h_bm.to("cuda")
    b_enc, b_dec = algorithmic_bytes(S, k, m, bs)
    b_dec *= args.lost  # each lost block: k/m - 1 survivors + parity read, 1 block written

    def time_it(fn):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.iters + 1)]
        fn(0)
        ev[0].record(s)
        for i in range(args.iters):
            fn(i + 1)
            ev[i + 1].record(s)
        torch.cuda.synchronize()
        return [ev[i].elapsed_time(ev[i + 1]) for i in range(args.iters)]

    variants = {}
    for t, u, g, nt, o in itertools.product(map(int, args.threads.split(",")),
                                            map(int, args.unroll.split(",")),
                                            map(int, args.grid.split(",")),
                                            map(int, args.nt.split(",")),
                                            map(int, args.occ.split(","))):
        variants[f"t{t}_u{u}_g{g}_nt{nt}" + (f"_o{o}" if o else "")] = (t, u, g, nt, o)

    # references on the same byte volume
    big = sets[0][0]
    copy_dst = torch.empty_like(big)
    half = big.numel() // 2
    xor_out = torch.empty(half, dtype=torch.uint8, device="cuda")

    results = {name: {"enc": [], "dec": []} for name in variants}
    results["torch_copy"] = {"GBps": []}
    results["torch_xor2"] = {"GBps": []}
    for _ in range(args.rounds):
        for name, (t, u, g, nt, o) in variants.items():
            assert xec.set_launch(u, g, nt, t) == 0
            assert xec.set_occupancy(o) == 0
            results[name]["enc"] += time_it(
                lambda i: xec.encode(sets[i % 2][0], sets[i % 2][1], S, bs, k, m, s))
            results[name]["dec"] += time_it(
                lambda i: xec.decode(sets[i % 2][0], sets[i % 2][1], S, bs, k, m, h_bm, scratch, s))
        xec.set_launch(0, 0, 0, 0)
        xec.set_occupancy(0)
        t = time_it(lambda i: copy_dst.copy_(big))
        results["torch_copy"]["GBps"] += [2 * big.numel() / (x * 1e-3) / 1e9 for x in t]
        t = time_it(lambda i: torch.bitwise_xor(big[:half // 2 * 2][:half], big[half:half * 2],
                                                out=xor_out))
        results["torch_xor2"]["GBps"] += [3 * half / (x * 1e-3) / 1e9 for x in t]

    summary = {"workload": args.workload, "k": k, "m": m, "bs": bs, "S": S, "lost": args.lost,
               "b_enc": b_enc, "b_dec": b_dec, "variants": {}}
    for name, r in results.items():
        if "enc" in r:
            e, d = statistics.median(r["enc"]), statistics.median(r["dec"])
            summary["variants"][name] = {
                "enc_ms_med": round(e, 4), "enc_ms_min": round(min(r["enc"]), 4),
                "enc_GBps": round(b_enc / (e * 1e-3) / 1e9, 1),
                "dec_ms_med": round(d, 4), "dec_GBps": round(b_dec / (d * 1e-3) / 1e9, 1)}
        else:
            summary["variants"][name] = {"GBps_med": round(statistics.median(r["GBps"]), 1),
                                         "GBps_max": round(max(r["GBps"]), 1)}
    for name, v in sorted(summary["variants"].items()):
        print(name, v)
    if args.out:
        Path(args.out).write_text(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
