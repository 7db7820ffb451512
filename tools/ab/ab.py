#!/usr/bin/env python3
"""In-process A/B of two or more builds of libxec_hip.so (tools/ab/build_rev.sh)
on one MI355X: same buffers, interleaved rounds, HIP events on the launching
stream -- so box-to-box spread (±3-4 %) cannot masquerade as a kernel change.

    python tools/ab/ab.py --libs base,new --workload cfg4 [--rounds 7 --iters 10]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))

from bench import WORKLOADS, algorithmic_bytes, erasure_pattern  # noqa: E402


def load(name: str):
    L = ctypes.CDLL(str(ROOT / "tools" / "ab" / f"libxec_{name}.so"))
    sz, vp = ctypes.c_size_t, ctypes.c_void_p
    L.xec_init.argtypes = [ctypes.c_int]
    L.xec_encode.argtypes = [vp, vp, sz, sz, sz, sz, vp]
    L.xec_decode.argtypes = [vp, vp, sz, sz, sz, sz, vp, vp, vp]
    assert L.xec_init(0) == 0
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--workload", default="cfg3",
                    help="bench.py workload name, or k,m,bs,S")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--occ", default="",
                    help="comma list of xec_set_occupancy values to cross with --libs "
                         "(0 = automatic, 8 = none); default: each lib's default only")
    ap.add_argument("--lost", type=int, default=1, help="lost data blocks per stripe (1..m)")
    ap.add_argument("--tiling", type=int, default=0,
                    help="xec_set_decode_tiling for every lib (0 = automatic)")
    ap.add_argument("--pattern", default="rotating", choices=["rotating", "same", "random"],
                    help="which data block a stripe loses (--lost 1 only): bench.py's "
                         "(7c) mod k, block 0 everywhere (one failed device), or seeded random")
    ap.add_argument("--launch", default="",
                    help="unroll,block_threads for xec_set_launch on every lib (default: none)")
    ap.add_argument("--variants", default="",
                    help="semicolon list of unroll,block_threads,occupancy launch variants to "
                         "cross with --libs in the same process (0,0,0 = the library's default)")
    ap.add_argument("--rotations", default="",
                    help="comma list of xec_set_rotation values to cross with --libs "
                         "(-1 none, 0 automatic, > 0 KiB per stripe); default: each lib's own")
    ap.add_argument("--tilings", default="",
                    help="comma list of xec_set_decode_tiling values to cross with --libs in "
                         "the same process (0 automatic, 1 stripe, 2 class, 3 work list)")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the identical-results check (diagnostic builds that store elsewhere)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import numpy as np
    import torch

    import xec  # for the shared fill; torch first, so all libs share its HIP runtime

    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    loaded = {n: load(n) for n in args.libs.split(",")}
    for L in loaded.values():
        if args.launch:
            u, t = (int(x) for x in args.launch.split(","))
            assert L.xec_set_launch(u, 0, 0, t) == 0
        if hasattr(L, "xec_set_decode_tiling"):  # round-1 builds predate the call
            assert L.xec_set_decode_tiling(args.tiling) == 0
        else:
            assert args.tiling == 0, "--tiling needs xec_set_decode_tiling"
    occs = [int(x) for x in args.occ.split(",")] if args.occ else [None]
    libs = {}
    for n, L in loaded.items():
        if args.variants:
            for v in args.variants.split(";"):
                u, t, o = (int(x) for x in v.split(","))
                libs[f"{n}@u{u}t{t}o{o}"] = (L, (u, t, o))
            continue
        if args.tilings:
            for t in (int(x) for x in args.tilings.split(",")):
                libs[f"{n}@t{t}"] = (L, ("til", t))
            continue
        if args.rotations:
            for r in (int(x) for x in args.rotations.split(",")):
                libs[f"{n}@r{r}"] = (L, ("rot", r))
            continue
        for o in occs:
            libs[n if o is None else f"{n}@o{o}"] = (L, o)
    if args.workload in WORKLOADS:
        k, m, bs, S, _ = WORKLOADS[args.workload]
    else:
        k, m, bs, S = (int(x) for x in args.workload.split(","))
    s = torch.cuda.current_stream()
    sh = ctypes.c_void_p(s.cuda_stream)
    sets = []
    for i in range(2):
        d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
        p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
        assert xec.fill_splitmix64(d, S, k * bs, 1896 + 7919 * i, s) == 0
        sets.append((d, p))
    bm = erasure_pattern(np, S, k, m, args.lost)
    if args.pattern != "rotating":
        assert args.lost == 1, "--pattern needs --lost 1"
        bm[:] = 1
        lost = (np.zeros(S, dtype=np.int64) if args.pattern == "same"
                else np.random.default_rng(1896).integers(0, k, S))
        bm[np.arange(S), lost] = 0
    h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
    scratch = h_bm.to("cuda")
    b_enc, b_dec = algorithmic_bytes(S, k, m, bs)
    b_dec *= args.lost

    # every build must produce the same parity and the same rebuilt data
    ref = None
    def use(L, o):
        if isinstance(o, tuple) and o[0] == "til":
            assert L.xec_set_decode_tiling(o[1]) == 0
        elif isinstance(o, tuple) and o[0] == "rot":
            assert L.xec_set_rotation(o[1]) == 0
        elif isinstance(o, tuple):
            assert L.xec_set_launch(o[0], 0, 0, o[1]) == 0
            assert L.xec_set_occupancy(o[2]) == 0
        elif o is not None:
            assert L.xec_set_occupancy(o) == 0
        return L

    for n, (L, o) in libs.items():
        use(L, o)
        d, p = sets[0]
        assert L.xec_encode(d.data_ptr(), p.data_ptr(), S, bs, k, m, sh) == 0
        assert L.xec_decode(d.data_ptr(), p.data_ptr(), S, bs, k, m, h_bm.data_ptr(),
                            scratch.data_ptr(), sh) == 0
        torch.cuda.synchronize()
        got = (p.clone(), d.clone())
        if ref is None:
            ref = got
        assert args.no_check or (torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])), n
    del ref, got

    def run(fn):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.iters + 1)]
        fn(0)
        ev[0].record(s)
        for i in range(args.iters):
            fn(i + 1)
            ev[i + 1].record(s)
        torch.cuda.synchronize()
        return [ev[i].elapsed_time(ev[i + 1]) for i in range(args.iters)]

    res = {n: {"enc": [], "dec": []} for n in libs}
    for _ in range(args.rounds):
        for n, (L, o) in libs.items():
            use(L, o)
            res[n]["enc"] += run(lambda i, L=L: L.xec_encode(
                sets[i % 2][0].data_ptr(), sets[i % 2][1].data_ptr(), S, bs, k, m, sh))
            res[n]["dec"] += run(lambda i, L=L: L.xec_decode(
                sets[i % 2][0].data_ptr(), sets[i % 2][1].data_ptr(), S, bs, k, m,
                h_bm.data_ptr(), scratch.data_ptr(), sh))
    out = {"workload": args.workload, "k": k, "m": m, "bs": bs, "S": S, "lost": args.lost,
           "pattern": args.pattern, "launch": args.launch, "libs": {}}
    for n, r in res.items():
        e, d = statistics.median(r["enc"]), statistics.median(r["dec"])
        out["libs"][n] = {"enc_ms_med": round(e, 4), "enc_GBps": round(b_enc / e / 1e6, 1),
                          "dec_ms_med": round(d, 4), "dec_GBps": round(b_dec / d / 1e6, 1)}
        print(n, out["libs"][n], flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
