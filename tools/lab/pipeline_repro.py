#!/usr/bin/env python3
"""Where does a pipeline decode go wrong?  Runs xec_pipeline encode + erase +
decode over a small grid of shapes with host buffers pinned or pageable, under
XEC_PIPELINE_STAGE_OPTS / XEC_PIPELINE_COPY_THREADS given per run, and for a
wrong decode prints which chunks, stripes and blocks differ from the original
(and whether the wrong bytes are zeros, i.e. the erased content, or stale
data) -- the hint to which copy overtook which.

    python tools/lab/pipeline_repro.py --opts ae,e --shapes 4,2,4096,25840,16,1 [--pattern parity]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opts", default="ae,e")
    ap.add_argument("--threads", default="4")
    ap.add_argument("--shapes", nargs="*", default=["4,2,4096,25840,16,1"])
    ap.add_argument("--pattern", default="one",
                    choices=["one", "every3", "sparse", "uniform", "skewed", "parity"],
                    help="one / every3 / sparse here, or a tools/fuzz_big.py loss_pattern kind")
    ap.add_argument("--encode-first", action="store_true",
                    help="as tools/fuzz_big.py --pipeline: the same pipeline encodes the host "
                         "batch (parity into a zeroed host buffer) before the decode")
    ap.add_argument("--seeds", default="5", help="comma list of pattern seeds")
    ap.add_argument("--mem", default="pageable", choices=["pageable", "pinned", "data", "parity"])
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import numpy as np
    import torch

    import xec

    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    s = torch.cuda.current_stream()
    sys.path.insert(0, str(ROOT / "tools"))
    from fuzz_big import loss_pattern
    for shape, seed in [(sh, int(sd)) for sh in args.shapes for sd in args.seeds.split(",")]:
        rng = np.random.default_rng(seed)
        k, m, bs, S, chunk, ns = (int(x) for x in shape.split(","))
        d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
        p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
        assert xec.fill_splitmix64(d, S, k * bs, 777, s) == 0
        assert xec.encode(d, p, S, bs, k, m, s) == 0
        ref_d, ref_p = d.cpu().numpy(), p.cpu().numpy()
        del d, p
        bm = np.ones((S, k + m), np.uint8)
        if args.pattern in ("uniform", "skewed", "parity"):
            bm = loss_pattern(np, rng, S, k, m, args.pattern)
        elif args.pattern == "one":
            bm[np.arange(S), rng.integers(0, k, S)] = 0
        elif args.pattern == "every3":
            c = np.arange(0, S, 3)
            bm[c, rng.integers(0, k, c.size)] = 0
        else:
            c = np.arange(0, S, 9)
            bm[c, rng.integers(0, k, c.size)] = 0
        for opts in args.opts.split(","):
            for th in args.threads.split(","):
                os.environ["XEC_PIPELINE_STAGE_OPTS"] = opts
                os.environ["XEC_PIPELINE_COPY_THREADS"] = th
                pin_d = args.mem in ("pinned", "parity")
                pin_p = args.mem in ("pinned", "data")

                def host(a, pin):
                    t = torch.from_numpy(a.copy())
                    return t.pin_memory() if pin else t

                for rep in range(args.reps):
                    h_d, h_p = host(ref_d, pin_d), host(ref_p, pin_p)
                    hv = h_d.numpy().reshape(S, k, bs)
                    h_bm = torch.from_numpy(bm.reshape(-1).copy()).pin_memory()
                    enc_ok = None
                    with xec.Pipeline(chunk, bs, k, m, ns) as pl:
                        if args.encode_first:
                            h_p.zero_()
                            enc_ok = pl.encode(h_d, h_p, S) == 0 and bool(
                                np.array_equal(h_p.numpy(), ref_p))
                        hv[bm[:, :k] == 0] = 0
                        st = int(pl.decode(h_d, h_p, S, h_bm))
                    got = h_d.numpy().reshape(S, k, bs)
                    want = ref_d.reshape(S, k, bs)
                    bad = np.argwhere((got != want).any(axis=2))
                    row = {"shape": shape, "seed": seed, "opts": opts, "threads": th, "rep": rep,
                           "status": st, "encode_ok": enc_ok, "bad_blocks": int(len(bad)),
                           "parity_intact": bool(np.array_equal(h_p.numpy(), ref_p))}
                    if len(bad):
                        lost = bm[bad[:, 0], bad[:, 1]] == 0
                        zeros = [(got[c, i] == 0).all() for c, i in bad[:50]]
                        row.update({"first_bad": bad[:8].tolist(),
                                    "bad_chunks": sorted(set((bad[:, 0] // chunk).tolist()))[:20],
                                    "n_bad_chunks": len(set((bad[:, 0] // chunk).tolist())),
                                    "bad_were_lost": int(lost.sum()),
                                    "bad_all_zero_first50": int(sum(zeros))})
                    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
