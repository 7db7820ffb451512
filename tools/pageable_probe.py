#!/usr/bin/env python3
"""How fast does the host-in / host-out path run from PAGEABLE host memory?

The north star's batch starts and ends in "file / socket buffers", which are
ordinary (pageable) memory unless the caller pins them.  xec_pipeline
(csrc/xec_pipeline.cpp) hands the caller's pointers to hipMemcpyAsync; for
pageable memory HIP stages the copy itself.  Measured on one MI355X, 1 GiB of
data at config 3's shape, best of --reps:
  * raw H2D / D2H of the batch, pinned and pageable;
  * xec_pipeline encode / decode with pinned and with pageable buffers
    (both checked bit-exact against a device encode).
Data GB/s (reference convention).

    python tools/pageable_probe.py [--stripes 64] [--reps 3] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))
sys.path.insert(0, str(ROOT))

from bench import HOST_CHUNK_STRIPES, HOST_STREAMS, erasure_pattern  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=64)
    ap.add_argument("--shape", default="16,1,1048576",
                    help="k,m,bs (default config 3's; config 4: 32,1,4096 with --stripes 8192 "
                         "--chunk 1024)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--chunk", type=int, default=HOST_CHUNK_STRIPES)
    ap.add_argument("--streams", type=int, default=HOST_STREAMS)
    ap.add_argument("--kinds", default="pinned,pageable",
                    help="comma list of: pinned, pageable, data_pageable_parity_pinned, "
                         "data_pinned_parity_pageable")
    ap.add_argument("--copy-threads", default="",
                    help="comma list of XEC_PIPELINE_COPY_THREADS values to A/B in one "
                         "process (each pipeline reads it at create; 0 = HIP stages pageable "
                         "inputs); default: the library's")
    ap.add_argument("--rounds", type=int, default=1,
                    help="repeat the kinds x copy-threads sweep, interleaved")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import numpy as np
    import torch

    import xec

    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    k, m, bs = (int(x) for x in args.shape.split(","))
    S = args.stripes
    nbytes = S * k * bs
    s = torch.cuda.current_stream()
    d_d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    d_p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
    assert xec.fill_splitmix64(d_d, S, k * bs, 1896, s) == 0
    assert xec.encode(d_d, d_p, S, bs, k, m, s) == 0
    ref_d, ref_p = d_d.cpu(), d_p.cpu()
    bm = erasure_pattern(np, S, k, m)
    h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
    out = {"shape": f"k={k}+{m}, {bs >> 10} KiB x {S} stripes ({nbytes >> 20} MiB data)",
           "library": xec.build_info(),
           "pipeline": f"{args.chunk}-stripe chunks x {args.streams} streams"}

    def best(fn, before=None):
        ts = []
        for _ in range(args.reps + 1):
            if before:
                before()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return min(ts[1:])

    # (data, parity) buffers: pinned or pageable each; the mixed pairs say
    # which buffer a pageable slowdown comes from
    kinds = {"pinned": (True, True), "pageable": (False, False),
             "data_pageable_parity_pinned": (False, True),
             "data_pinned_parity_pageable": (True, False)}
    threads = args.copy_threads.split(",") if args.copy_threads else [None]
    sweep = [(kind, th) for _ in range(args.rounds) for kind in kinds
             if kind in args.kinds.split(",") for th in threads]
    for kind, th in sweep:
        pin_d, pin_p = kinds[kind]
        if th is not None:  # "8" or "8:af" (XEC_PIPELINE_STAGE_OPTS letters)
            n_th, sep, opts = th.partition(":")
            os.environ["XEC_PIPELINE_COPY_THREADS"] = n_th
            if sep:
                os.environ["XEC_PIPELINE_STAGE_OPTS"] = opts
            else:
                os.environ.pop("XEC_PIPELINE_STAGE_OPTS", None)
        h_d = torch.empty(nbytes, dtype=torch.uint8)
        h_p = torch.zeros(S * m * bs, dtype=torch.uint8)
        if pin_d:
            h_d = h_d.pin_memory()
        if pin_p:
            h_p = h_p.pin_memory()
        h_d.copy_(ref_d)
        r = {}
        r["h2d_GBps"] = round(nbytes / best(lambda: d_d.copy_(h_d, non_blocking=True)) / 1e9, 2)
        r["d2h_GBps"] = round(nbytes / best(lambda: h_d.copy_(d_d, non_blocking=True)) / 1e9, 2)
        h_d.copy_(ref_d)
        pl = xec.Pipeline(args.chunk, bs, k, m, args.streams)
        rcs = []
        t = best(lambda: rcs.append(int(pl.encode(h_d, h_p, S))))
        r["pipeline_encode_GBps_data"] = round(nbytes / t / 1e9, 2)
        r["encode_bit_exact"] = bool(torch.equal(h_p, ref_p)) and not any(rcs)
        hv = h_d.numpy().reshape(S, k, bs)

        def erase():
            hv[bm[:, :k] == 0] = 0

        t = best(lambda: rcs.append(int(pl.decode(h_d, h_p, S, h_bm))), before=erase)
        r["pipeline_decode_GBps_data"] = round(nbytes / t / 1e9, 2)
        r["decode_bit_exact"] = bool(torch.equal(h_d, ref_d)) and not any(rcs)
        pl.close()
        name = kind if th is None else f"{kind}/threads{th}"
        if args.rounds > 1:
            out.setdefault(name, []).append(r)
        else:
            out[name] = r
        print(name, r, flush=True)
        del h_d, h_p, hv
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
