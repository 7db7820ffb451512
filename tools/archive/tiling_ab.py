#!/usr/bin/env python3
"""In-process A/B of the decode tilings (xec_set_decode_tiling) on one MI355X.

For each shape and each number of lost data blocks per stripe (one per class,
bench.erasure_pattern), times xec_decode with stripe tiles (1), class tiles (2),
work-list tiles (3) and the automatic choice (0) -- with --device also
xec_decode_device and xec_decode_device_list -- in interleaved rounds on the
same buffers (three
rotating buffer sets, HIP events on the launching stream), and checks every
variant rebuilt the erased blocks bit-exactly (against a fresh device fill).
Also times encode on the same buffers as the reference point.  Rates are
algorithmic GB/s: decode (lost data blocks)*(k/m+1)*bs, encode S*(k+m)*bs per
launch.  --pattern sparse keeps the losses of only every 9th stripe, skew only
every 5th (the others lose nothing); --pattern fraction keeps them on a
fraction --fraction of the stripes, spread evenly over the batch (stripe c
keeps its losses when frac(c * 0.618...) < f): the sweep that prices the
work-list threshold (xec_api.cpp kListStripesNum / kListStripesDen).

    python tools/archive/tiling_ab.py [--shapes 16,2,1048576,256:16,8,65536,16384]
                              [--pattern uniform|sparse|skew] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))

from bench import algorithmic_bytes, erasure_pattern  # noqa: E402

DEFAULT_SHAPES = "16,2,1048576,256:16,8,65536,16384:32,8,65536,8192:16,4,65536,16384:8,2,1048576,256"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=DEFAULT_SHAPES)
    ap.add_argument("--lost", default="", help="comma list; default 1, m/2, m (distinct)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--occ", default="",
                    help="comma list of xec_set_occupancy values (1..8) to also time class "
                         "tiles at (variants class@oN); default: automatic residency only")
    ap.add_argument("--only-class", action="store_true",
                    help="time class tiles (and their --occ variants) and encode only")
    ap.add_argument("--pattern", default="uniform",
                    choices=["uniform", "sparse", "skew", "fraction"])
    ap.add_argument("--fraction", default="0.5",
                    help="--pattern fraction: comma list of stripe fractions that lose blocks")
    ap.add_argument("--variants", default="", help="comma list to keep (e.g. class,list)")
    ap.add_argument("--device", action="store_true",
                    help="also time the device-resident decodes: xec_decode_device (dev) and "
                         "xec_decode_device_list (devlist), bitmap already in HBM")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import numpy as np
    import torch

    import xec

    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    stream = torch.cuda.current_stream()
    results = []
    for shape in args.shapes.split(":"):
        k, m, bs, S = (int(x) for x in shape.split(","))
        losts = ([int(x) for x in args.lost.split(",")] if args.lost
                 else sorted({1, max(1, m // 2), m}))
        sets = []
        for s in range(3):
            d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
            p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
            assert xec.fill_splitmix64(d, S, k * bs, 1000 + s * 7919, stream) == 0
            assert xec.encode(d, p, S, bs, k, m, stream) == 0
            sets.append((d, p))
        b_enc, _ = algorithmic_bytes(S, k, m, bs)
        fracs = ([float(x) for x in args.fraction.split(",")] if args.pattern == "fraction"
                 else [None])
        for lost, frac in ((lo, f) for lo in losts for f in fracs):
            if lost > m:
                continue
            bm = erasure_pattern(np, S, k, m, lost)
            if args.pattern == "fraction":
                keep = (np.arange(S) * 0.6180339887498949) % 1.0 < frac
                bm[~keep] = 1
            elif args.pattern != "uniform":
                keep = np.arange(S) % (9 if args.pattern == "sparse" else 5) == 0
                bm[~keep] = 1
            lost_blocks = int((bm[:, :k] == 0).sum())
            h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
            d_bm = h_bm.to("cuda")
            scratch = [torch.empty_like(d_bm) for _ in range(3)]
            # variant -> (tiling, occupancy); occupancy None = automatic
            variants = ({"stripe": (1, None), "class": (2, None), "list": (3, None),
                         "auto": (0, None)} if m > 1
                        else {"stripe": (1, None), "list": (3, None)})
            if args.only_class and m > 1:
                variants = {"class": (2, None)}
            for o in (int(x) for x in args.occ.split(",") if x):
                variants[f"class@o{o}"] = (2 if m > 1 else 1, o)
            if args.device:
                variants["dev"] = (0, None)
                variants["devlist"] = (0, None)
            d_status = torch.zeros((1,), dtype=torch.int32, device="cuda")
            wbytes = xec.device_list_bytes(S, k, m)
            work = torch.empty((wbytes // 4,), dtype=torch.int32, device="cuda")

            def run_decode(v, d, p, scr):
                if v == "dev":
                    return xec.decode_device(d, p, S, bs, k, m, d_bm, d_status, stream)
                if v == "devlist":
                    return xec.decode_device_list(d, p, S, bs, k, m, d_bm, work, wbytes,
                                                  d_status, stream)
                return xec.decode(d, p, S, bs, k, m, h_bm, scr, stream)

            if args.variants:
                keep = set(args.variants.split(","))
                variants = {v: t for v, t in variants.items() if v in keep}
            times = {v: [] for v in variants}
            times["encode"] = []
            it = 0
            for _ in range(args.rounds):
                for v, t in list(variants.items()) + [("encode", None)]:
                    if t is not None:
                        assert xec.set_decode_tiling(t[0]) == 0
                        assert xec.set_occupancy(t[1] or 0) == 0
                    else:
                        assert xec.set_occupancy(0) == 0
                    evs = [(torch.cuda.Event(enable_timing=True),
                            torch.cuda.Event(enable_timing=True)) for _ in range(args.iters)]
                    for i in range(args.iters):
                        d, p = sets[it % 3]
                        it += 1
                        evs[i][0].record(stream)
                        if v == "encode":
                            assert xec.encode(d, p, S, bs, k, m, stream) == 0
                        else:
                            assert run_decode(v, d, p, scratch[it % 3]) == 0
                        evs[i][1].record(stream)
                    torch.cuda.synchronize()
                    times[v] += [a.elapsed_time(b) for a, b in evs]
            # correctness of each variant: erase -> decode -> == fresh fill
            fresh = torch.empty_like(sets[0][0])
            ok = {}
            for v, t in variants.items():
                assert xec.set_decode_tiling(t[0]) == 0
                assert xec.set_occupancy(t[1] or 0) == 0
                d, p = sets[0]
                assert xec.erase(d, p, S, bs, k, m, d_bm, stream) == 0
                assert run_decode(v, d, p, scratch[0]) == 0
                assert xec.fill_splitmix64(fresh, S, k * bs, 1000, stream) == 0
                ok[v] = bool(torch.equal(fresh, d)) and int(d_status.item()) == 0
            assert xec.set_decode_tiling(0) == 0
            assert xec.set_occupancy(0) == 0
            del fresh
            b_dec = lost_blocks * (k // m + 1) * bs
            row = {"k": k, "m": m, "bs": bs, "S": S, "pattern": args.pattern,
                   "stripe_fraction": frac,
                   "stripes_lost": int((bm[:, :k] == 0).any(axis=1).sum()),
                   "lost_per_stripe": lost, "lost_blocks": lost_blocks,
                   "class_fraction": lost / m, "bit_exact": ok}
            for v, ts in times.items():
                med = statistics.median(ts)
                b = b_enc if v == "encode" else b_dec
                row[v] = {"median_ms": round(med, 4), "GBps": round(b / med / 1e6, 1),
                          "frac_8TBps": round(b / med / 1e6 / 8000, 4)}
            print(json.dumps(row), flush=True)
            results.append(row)
        del sets
        torch.cuda.empty_cache()
    if args.out:
        Path(args.out).write_text(json.dumps(results, indent=1) + "\n")


if __name__ == "__main__":
    main()
