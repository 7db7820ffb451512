#!/usr/bin/env python3
"""Residency at finer steps than whole waves per SIMD: times the product
encode/decode of an XEC_LDS_BYTES-aware build (tools/archive/ab/patches/
lds_env_override.py, built as tools/ab/libxec_ldsenv.so) for several LDS
reservations per workgroup, interleaved in one process.

    python tools/archive/ab/lds_sweep.py --workload cfg3 --lds 0,20480,16384,13312
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))

from bench import algorithmic_bytes, erasure_pattern, workload_shape  # noqa: E402
from tools.ab.ab import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--lds", default="0,20480,18176,16384,14848,13312")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import numpy as np
    import torch

    import xec

    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    L = load("ldsenv")
    k, m, bs, S, _ = workload_shape(args.workload)
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    sets = []
    for i in range(2):
        d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
        p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
        assert xec.fill_splitmix64(d, S, k * bs, 1896 + 7919 * i, s) == 0
        sets.append((d, p))
    h_bm = torch.from_numpy(erasure_pattern(np, S, k, m).reshape(-1)).pin_memory()
    scratch = h_bm.to("cuda")
    b_enc, b_dec = algorithmic_bytes(S, k, m, bs)

    def run(fn):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.iters + 1)]
        fn(0)
        ev[0].record(s)
        for i in range(args.iters):
            fn(i + 1)
            ev[i + 1].record(s)
        torch.cuda.synchronize()
        return [ev[i].elapsed_time(ev[i + 1]) for i in range(args.iters)]

    vals = [int(x) for x in args.lds.split(",")]
    res = {v: {"enc": [], "dec": []} for v in vals}
    for _ in range(args.rounds):
        for v in vals:
            if v:
                os.environ["XEC_LDS_BYTES"] = str(v)
            else:
                os.environ.pop("XEC_LDS_BYTES", None)  # the library's own choice
            res[v]["enc"] += run(lambda i: L.xec_encode(sets[i % 2][0].data_ptr(),
                                                        sets[i % 2][1].data_ptr(), S, bs, k, m, sh))
            res[v]["dec"] += run(lambda i: L.xec_decode(
                sets[i % 2][0].data_ptr(), sets[i % 2][1].data_ptr(), S, bs, k, m,
                h_bm.data_ptr(), scratch.data_ptr(), sh))
    os.environ.pop("XEC_LDS_BYTES", None)
    out = {"workload": args.workload, "results": {}}
    for v in vals:
        e, d = statistics.median(res[v]["enc"]), statistics.median(res[v]["dec"])
        name = "default" if v == 0 else f"{v}B_{163840 // v}wg_per_cu"
        out["results"][name] = {"enc_GBps": round(b_enc / e / 1e6, 1),
                                "dec_GBps": round(b_dec / d / 1e6, 1)}
        print(name, out["results"][name], flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
