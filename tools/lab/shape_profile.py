#!/usr/bin/env python3
"""One shape's encode and one loss pattern's decode, repeated, for rocprofv3
(32+4 x 1 MiB).  Run under rocprofv3 --kernel-trace --stats
(timed launches) or --pmc FETCH_SIZE / WRITE_SIZE (HBM bytes): every launch of
the encode kernel and of the decode kernel has the same shape and bytes, so
the per-kernel averages are the shape's.

Patterns (one decode bitmap for the whole run):
  select   -- the reference's draw: select_lost_blocks(k, m, lost=m) per stripe
              (utils.cpp:100-127, seeded: xec_select_lost_blocks), data AND
              parity blocks, one per class
  random1  -- one uniformly random data block per stripe
  same     -- data block 0 of every stripe (one failed device)
  rotating -- data block (7c) mod k (bench.py's pattern)

Decoding in place again rebuilds the same bytes (the lost blocks were rebuilt
by the first decode; the kernel reads only survivors and parity), so the
decode repeats without re-erasing.  The rebuild is checked exact once.  Prints
a JSON line with HIP-event medians and the decode's algorithmic bytes.

    python tools/lab/shape_profile.py --shape 32,4,1048576,256 --pattern select
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


def bitmap(np, xec, pattern, S, k, m, seed):
    bm = np.ones((S, k + m), dtype=np.uint8)
    c = np.arange(S)
    if pattern == "select":
        for s in range(S):
            row = np.ascontiguousarray(bm[s])
            assert xec.select_lost_blocks(k, m, m, row, seed + s) == 0
            bm[s] = row
    elif pattern == "random1":
        bm[c, np.random.default_rng(seed).integers(0, k, S)] = 0
    elif pattern == "same":
        bm[:, 0] = 0
    elif pattern == "rotating":
        bm[c, (7 * c) % k] = 0
    else:
        raise SystemExit(f"unknown pattern {pattern}")
    return bm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="32,4,1048576,256", help="k,m,bs,S")
    ap.add_argument("--pattern", default="select")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--seed", type=int, default=1896)
    ap.add_argument("--rotation", type=int, default=0, help="xec_set_rotation (0 automatic)")
    ap.add_argument("--occ", default="",
                    help="comma list of xec_set_occupancy values timed in interleaved rounds "
                         "(0 automatic, 8 no cap); default: the automatic choice only")
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch

    import xec

    k, m, bs, S = (int(x) for x in args.shape.split(","))
    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    assert xec.set_rotation(args.rotation) == 0
    s = torch.cuda.current_stream()
    d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
    p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
    fresh = torch.empty_like(d)
    assert xec.fill_splitmix64(d, S, k * bs, args.seed, s) == 0
    assert xec.fill_splitmix64(fresh, S, k * bs, args.seed, s) == 0
    bm = bitmap(np, xec, args.pattern, S, k, m, args.seed)
    h = torch.from_numpy(bm.reshape(-1)).pin_memory()
    dbm = h.to("cuda")
    scratch = torch.empty_like(dbm)
    lost_data = int((bm[:, :k] == 0).sum())
    assert xec.encode(d, p, S, bs, k, m, s) == 0
    assert xec.erase(d, p, S, bs, k, m, dbm, s) == 0
    assert xec.decode(d, p, S, bs, k, m, h, scratch, s) == 0
    exact = bool(torch.equal(d, fresh))
    del fresh
    tiling = xec.DECODE_KERNELS.get(xec.decode_tiling_used(), "?")

    def run(fn):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.iters + 1)]
        fn()
        ev[0].record(s)
        for i in range(args.iters):
            fn()
            ev[i + 1].record(s)
        torch.cuda.synchronize()
        return statistics.median(ev[i].elapsed_time(ev[i + 1]) for i in range(args.iters))

    b_enc = S * (k + m) * bs
    b_dec = lost_data * (k // m + 1) * bs  # each rebuild reads k/m blocks, writes 1
    if args.occ:  # residency A/B: every value timed in each round, rounds interleaved
        occs = [int(x) for x in args.occ.split(",")]
        te = {o: [] for o in occs}
        td = {o: [] for o in occs}
        for _ in range(args.rounds):
            for o in occs:
                assert xec.set_occupancy(o) == 0
                te[o].append(run(lambda: xec.encode(d, p, S, bs, k, m, s)))
                td[o].append(run(lambda: xec.decode(d, p, S, bs, k, m, h, scratch, s)))
        assert xec.set_occupancy(0) == 0
        for o in occs:
            e, dd = statistics.median(te[o]), statistics.median(td[o])
            print(json.dumps({"shape": args.shape, "pattern": args.pattern, "occupancy": o,
                              "encode_ms": round(e, 4), "encode_GBps": round(b_enc / e / 1e6, 1),
                              "decode_ms": round(dd, 4), "decode_GBps": round(b_dec / dd / 1e6, 1),
                              "decode_tiling": tiling, "exact": exact}), flush=True)
        return
    # the decode's parity stays as encode left it (decode never writes parity)
    te = run(lambda: xec.encode(d, p, S, bs, k, m, s))
    td = run(lambda: xec.decode(d, p, S, bs, k, m, h, scratch, s))
    print(json.dumps({"shape": args.shape, "pattern": args.pattern, "rotation": args.rotation,
                      "lost_data_blocks": lost_data, "decode_tiling": tiling, "exact": exact,
                      "encode_ms": round(te, 4), "encode_GBps": round(b_enc / te / 1e6, 1),
                      "decode_ms": round(td, 4), "decode_GBps": round(b_dec / td / 1e6, 1),
                      "encode_algorithmic_bytes": b_enc, "decode_algorithmic_bytes": b_dec,
                      "library": xec.build_info()}), flush=True)


if __name__ == "__main__":
    main()
