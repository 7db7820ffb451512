#!/usr/bin/env python3
"""Does WHICH block a stripe loses change the decode rate?

One lost data block per stripe, three patterns over the same batch:
  same      -- block 0 in every stripe: one failed device (the common case in
               a real system: the same shard index is gone from every stripe)
  same2     -- blocks 0 and 1 in every stripe (m >= 2): two failed devices
  rotating  -- block (7c) mod k: bench.py's pattern
  random    -- a seeded uniform block per stripe, like the reference's
               select_lost_blocks (src/utils/utils.cpp)
The decode reads the lost block's class (k/m - 1 data blocks + its parity)
and writes the lost block, so the bytes are the same for every pattern; only
their addresses differ.  Product xec_decode (automatic tiling), HIP events on
the launching stream, patterns interleaved over rounds; each pattern's
rebuild is checked against a fresh fill once.

With --rotations R1,R2,... every rotation (xec_set_rotation: -1 none, 0 the
library's automatic choice, > 0 chunks per stripe) is timed in the same
interleaved rounds, encode included, and each is checked exact.

    python tools/lab/loss_pattern_probe.py [--shapes 16,2,1048576,256 ...] [--rotations -1,3]
                                           [--out f.json]
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

from bench import algorithmic_bytes  # noqa: E402

DEFAULT_SHAPES = ["16,2,1048576,256", "8,2,1048576,256", "16,4,65536,16384",
                  "16,8,65536,16384", "32,8,65536,8192", "16,1,1048576,256"]


def patterns(np, S, k, m, seed):
    c = np.arange(S)
    rng = np.random.default_rng(seed)
    lost = {"same": np.zeros(S, dtype=np.int64), "rotating": (7 * c) % k,
            "random": rng.integers(0, k, S)}
    out = {}
    for name, idx in lost.items():
        bm = np.ones((S, k + m), dtype=np.uint8)
        bm[c, idx] = 0
        out[name] = bm
    if m >= 2:  # two failed devices: blocks 0 and 1 (two classes) gone from every stripe
        bm = np.ones((S, k + m), dtype=np.uint8)
        bm[:, 0] = 0
        bm[:, 1] = 0
        out["same2"] = bm
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="*", default=DEFAULT_SHAPES)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--seed", type=int, default=1896)
    ap.add_argument("--out", default="")
    ap.add_argument("--rotations", default="",
                    help="comma list of xec_set_rotation values to A/B in one process")
    ap.add_argument("--tiling", type=int, default=0,
                    help="xec_set_decode_tiling for every decode (0 = automatic)")
    args = ap.parse_args()
    import numpy as np
    import torch

    import xec

    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    assert xec.set_decode_tiling(args.tiling) == 0
    s = torch.cuda.current_stream()
    res = {"note": "tools/lab/loss_pattern_probe.py: xec_decode by loss pattern, one lost "
                   "data block per stripe; GB/s of algorithmic bytes", "shapes": {}}
    for shape in args.shapes:
        k, m, bs, S = (int(x) for x in shape.split(","))
        d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
        p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
        fresh = torch.empty_like(d)
        assert xec.fill_splitmix64(d, S, k * bs, args.seed, s) == 0
        assert xec.encode(d, p, S, bs, k, m, s) == 0
        b_enc, b_dec1 = algorithmic_bytes(S, k, m, bs)
        pats = patterns(np, S, k, m, args.seed)
        h = {n: torch.from_numpy(bm.reshape(-1)).pin_memory() for n, bm in pats.items()}
        dev = {n: t.to("cuda") for n, t in h.items()}
        scratch = torch.empty_like(next(iter(dev.values())))
        rots = [int(x) for x in args.rotations.split(",")] if args.rotations else [None]
        ok = {}
        for rot in rots:
            if rot is not None:
                assert xec.set_rotation(rot) == 0
            for n in pats:  # erase -> decode -> equal to a fresh fill
                assert xec.encode(d, p, S, bs, k, m, s) == 0
                assert xec.erase(d, p, S, bs, k, m, dev[n], s) == 0
                assert xec.decode(d, p, S, bs, k, m, h[n], scratch, s) == 0
                assert xec.fill_splitmix64(fresh, S, k * bs, args.seed, s) == 0
                ok[(rot, n)] = bool(torch.equal(d, fresh))
        del fresh

        def run(fn):
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.iters + 1)]
            fn()
            ev[0].record(s)
            for i in range(args.iters):
                fn()
                ev[i + 1].record(s)
            torch.cuda.synchronize()
            return [ev[i].elapsed_time(ev[i + 1]) for i in range(args.iters)]

        t = {(rot, n): [] for rot in rots for n in pats}
        t_enc = {rot: [] for rot in rots}
        for _ in range(args.rounds):
            for rot in rots:
                if rot is not None:
                    assert xec.set_rotation(rot) == 0
                t_enc[rot] += run(lambda: xec.encode(d, p, S, bs, k, m, s))
                for n in pats:
                    t[(rot, n)] += run(lambda n=n: xec.decode(d, p, S, bs, k, m, h[n], scratch, s))
        xec.set_rotation(0)
        out = {}
        for rot in rots:
            e = statistics.median(t_enc[rot])
            r = {"encode_ms": round(e, 4), "encode_GBps": round(b_enc / e / 1e6, 1),
                 "tiling": xec.DECODE_KERNELS.get(xec.decode_tiling_used(), "?")}
            for n in pats:
                md = statistics.median(t[(rot, n)])
                b_dec = b_dec1 * (2 if n == "same2" else 1)
                r[n] = {"ms": round(md, 4), "GBps": round(b_dec / md / 1e6, 1),
                        "exact": ok[(rot, n)]}
            out["default" if rot is None else f"rot{rot}"] = r
            print(shape, "default" if rot is None else f"rot{rot}", json.dumps(r), flush=True)
        res["shapes"][shape] = out if rots != [None] else out["default"]
        del d, p, scratch
        torch.cuda.empty_cache()
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
