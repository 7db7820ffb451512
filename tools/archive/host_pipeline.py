#!/usr/bin/env python3
"""End-to-end (host-in / host-out) XOR-EC rate on one MI355X: SURVEY.md §8(f) #1.

The batch starts and ends in pinned host memory.  Measured:
  * link     -- raw pinned H2D and D2H copy rates (the bound of this path);
  * serial   -- H2D whole batch, encode, D2H parity, one stream;
  * pipeline -- xec_pipeline_encode / _decode with chunking over N streams.
Rates are in the reference's convention (data bytes / s, GB = 1e9), the
natural unit for a path whose bytes cross PCIe once.

    python tools/archive/host_pipeline.py [--workload cfg3|k,m,bs,S] [--lost N] [--reps 3] [--out f.json]
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
sys.path.insert(0, str(ROOT))

from bench import erasure_pattern, workload_shape  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--chunks", default="4,8,16,32")
    ap.add_argument("--streams", default="2,3,4")
    ap.add_argument("--lost", type=int, default=1,
                    help="lost data blocks per stripe, one per class (bench.py erasure_pattern)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import numpy as np
    import torch

    import xec

    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    k, m, bs, S, _ = workload_shape(args.workload)
    data_bytes = S * k * bs
    h_d = torch.empty(data_bytes, dtype=torch.uint8).pin_memory()
    h_p = torch.empty(S * m * bs, dtype=torch.uint8).pin_memory()
    d_d = torch.empty(data_bytes, dtype=torch.uint8, device="cuda")
    d_p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    assert xec.fill_splitmix64(d_d, S, k * bs, 1896, s) == 0
    h_d.copy_(d_d)
    assert xec.encode(d_d, d_p, S, bs, k, m, s) == 0
    ref_p = d_p.cpu()
    bm = erasure_pattern(np, S, k, m, args.lost)
    h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
    torch.cuda.synchronize()

    def timed(fn):
        ts = []
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts)

    res = {"workload": args.workload, "k": k, "m": m, "bs": bs, "S": S, "lost": args.lost,
           "data_bytes": data_bytes, "lib": str(xec.LIB_PATH)}
    t = timed(lambda: d_d.copy_(h_d, non_blocking=True))
    res["link_h2d_GBps"] = round(data_bytes / t / 1e9, 2)
    t = timed(lambda: h_d.copy_(d_d, non_blocking=True))
    res["link_d2h_GBps"] = round(data_bytes / t / 1e9, 2)

    def serial():
        d_d.copy_(h_d, non_blocking=True)
        assert xec.encode(d_d, d_p, S, bs, k, m, s) == 0
        h_p.copy_(d_p, non_blocking=True)
    t = timed(serial)
    res["serial_encode_GBps"] = round(data_bytes / t / 1e9, 2)
    assert torch.equal(h_p, ref_p)

    best = None
    res["pipeline"] = []
    for ch in map(int, args.chunks.split(",")):
        for ns in map(int, args.streams.split(",")):
            with xec.Pipeline(ch, bs, k, m, ns) as pl:
                h_p.zero_()
                t_enc = timed(lambda: pl.encode(h_d, h_p, S))
                ok = bool(torch.equal(h_p, ref_p))
                t_dec = timed(lambda: pl.decode(h_d, h_p, S, h_bm))
            row = {"chunk_stripes": ch, "streams": ns, "encode_GBps": round(data_bytes / t_enc / 1e9, 2),
                   "decode_GBps": round(data_bytes / t_dec / 1e9, 2), "encode_bit_exact": ok}
            res["pipeline"].append(row)
            print(row, flush=True)
            if best is None or row["encode_GBps"] > best["encode_GBps"]:
                best = row
    # decode correctness at the best shape: erase on the host, rebuild, compare
    with xec.Pipeline(best["chunk_stripes"], bs, k, m, best["streams"]) as pl:
        ref_d = h_d.clone()
        hv = h_d.numpy().reshape(S, k, bs)
        hv[bm[:, :k] == 0] = 0
        assert pl.decode(h_d, h_p, S, h_bm) == 0
        res["decode_bit_exact"] = bool(torch.equal(h_d, ref_d))
    res["best"] = best
    print(json.dumps({k_: v for k_, v in res.items() if k_ != "pipeline"}))
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
