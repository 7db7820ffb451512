#!/usr/bin/env python3
"""Interleaved A/B of experimental encode variants (tools/lab/liblab.so) against
the product kernel, on one MI355X, HIP events on the launching stream.

    python tools/lab/lab.py [--rounds 7] [--iters 10] [--variants 0,1,...] [--gap-ms 0]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", default="")
    ap.add_argument("--S", type=int, default=256)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--bs", type=int, default=1 << 20)
    ap.add_argument("--gap-ms", type=float, default=0.0, help="host sleep between launches")
    ap.add_argument("--out", default="")
    ap.add_argument("--decode", action="store_true", help="time the decode diagnostics")
    ap.add_argument("--ceiling", action="store_true", help="time read/write/copy ceilings")
    ap.add_argument("--dec-sc1", action="store_true",
                    help="--decode: diagnostics store their result sc1 (the product's policy)")
    ap.add_argument("--wburst", action="store_true",
                    help="time write-only bursts of 1/4/16 KiB per workgroup, nt vs sc1")
    ap.add_argument("--wscatter", action="store_true",
                    help="time scattered write-only streams (the decode's rebuilt-block "
                         "pattern) against a dense one, nt and sc1")
    ap.add_argument("--occ", default="0", help="--ceiling: waves-per-SIMD caps (0 = none), "
                                               "crossed with the product encode's own setting")
    args = ap.parse_args()

    import torch

    import xec

    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    L = ctypes.CDLL(str(Path(__file__).resolve().parent / "liblab.so"))
    L.lab_variant_name.restype = ctypes.c_char_p
    L.lab_variant_name.argtypes = [ctypes.c_int]
    L.lab_encode.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_uint64] * 4 + [ctypes.c_void_p]
    names = {}
    v = 0
    while L.lab_variant_name(v):
        names[v] = L.lab_variant_name(v).decode()
        v += 1
    chosen = [int(x) for x in args.variants.split(",")] if args.variants else sorted(names)

    S, k, m, bs = args.S, args.k, 1, args.bs
    s = torch.cuda.current_stream()
    sh = s.cuda_stream
    sets = []
    for i in range(2):
        d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
        p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
        assert xec.fill_splitmix64(d, S, k * bs, 1896 + 7919 * i, s) == 0
        assert xec.encode(d, p, S, bs, k, m, s) == 0
        sets.append((d, p))
    torch.cuda.synchronize()
    ref = [p.clone() for _, p in sets]
    b_enc = S * (k + m) * bs

    if args.decode:
        return decode_lab(args, L, torch, xec, sets, S, k, m, bs, s, sh)
    if args.ceiling:
        return ceiling_lab(args, L, torch, xec, sets, S, k, m, bs, s, sh)
    if args.wburst:
        return wburst_lab(args, L, torch, sets, S, k, bs, s, sh)
    if args.wscatter:
        return wscatter_lab(args, L, torch, sets, S, k, bs, s, sh)

    # correctness of every variant first
    bad = []
    for v in chosen:
        for i, (d, p) in enumerate(sets):
            p.zero_()
            assert L.lab_encode(v, d.data_ptr(), p.data_ptr(), S, bs, k, m, sh) == 0
            torch.cuda.synchronize()
            if not torch.equal(p, ref[i]):
                bad.append(names[v])
    print("incorrect variants:", bad, flush=True)

    def run(fn):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.iters)]
        fn(0)
        ts = []
        for i in range(args.iters):
            if args.gap_ms:
                torch.cuda.synchronize()
                time.sleep(args.gap_ms * 1e-3)
            ev[2 * i].record(s)
            fn(i + 1)
            ev[2 * i + 1].record(s)
        torch.cuda.synchronize()
        return [ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(args.iters)]

    # --occ crosses every variant with residency caps: the product via
    # xec_set_occupancy, lab launches that honour g_ceiling_lds via the same LDS
    # reservation (only the grouped-tile variants do); 0 = product default / none
    L.lab_set_ceiling_lds.argtypes = [ctypes.c_uint32]
    occs = [int(x) for x in args.occ.split(",")]

    def lds(w):
        return 0 if w <= 0 or w >= 8 else ((160 * 1024) // (4 * w)) & ~511

    def tag(n, w):
        return n if len(occs) == 1 else f"{n}@o{w}"

    res = {tag(names[v], w): [] for w in occs for v in chosen}
    res.update({tag("product", w): [] for w in occs})
    for _ in range(args.rounds):
        for w in occs:
            assert xec.set_occupancy(w) == 0
            L.lab_set_ceiling_lds(lds(w))
            res[tag("product", w)] += run(
                lambda i: xec.encode(sets[i % 2][0], sets[i % 2][1], S, bs, k, m, s))
            for v in chosen:
                res[tag(names[v], w)] += run(lambda i, v=v: L.lab_encode(
                    v, sets[i % 2][0].data_ptr(), sets[i % 2][1].data_ptr(), S, bs, k, m, sh))
    xec.set_occupancy(0)
    L.lab_set_ceiling_lds(0)
    out = {}
    for n, ts in res.items():
        med = statistics.median(ts)
        out[n] = {"ms_med": round(med, 4), "ms_min": round(min(ts), 4),
                  "GBps_med": round(b_enc / (med * 1e-3) / 1e9, 1),
                  "GBps_best": round(b_enc / (min(ts) * 1e-3) / 1e9, 1)}
    for n, r in sorted(out.items(), key=lambda kv: -kv[1]["GBps_med"]):
        print(f"{n:24s} {r}")
    if args.out:
        Path(args.out).write_text(json.dumps({"shape": [S, k, m, bs], "gap_ms": args.gap_ms,
                                              "incorrect": bad, "results": out}, indent=1))



def decode_lab(args, L, torch, xec, sets, S, k, m, bs, s, sh):
    import numpy as np
    # --occ W (first value) caps the diagnostics' residency like the product's;
    # --dec-sc1 stores their result sc1 like the product's decode
    w = int(args.occ.split(",")[0])
    L.lab_set_ceiling_lds.argtypes = [ctypes.c_uint32]
    L.lab_set_ceiling_lds(0 if w <= 0 or w >= 8 else ((160 * 1024) // (4 * w)) & ~511)
    L.lab_set_dec_store_aux.argtypes = [ctypes.c_int]
    L.lab_set_dec_store_aux(16 if args.dec_sc1 else 2)
    L.lab_dec_name.restype = ctypes.c_char_p
    L.lab_dec_name.argtypes = [ctypes.c_int]
    L.lab_decode.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_uint64] * 4 + [ctypes.c_void_p]
    names = {}
    v = 0
    while L.lab_dec_name(v):
        names[v] = L.lab_dec_name(v).decode()
        v += 1
    lost = (7 * np.arange(S)) % k
    bm = np.ones((S, k + m), np.uint8)
    bm[np.arange(S), lost] = 0
    h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
    d_bm = h_bm.to("cuda")
    table = torch.from_numpy(lost.astype(np.uint8)).to("cuda")
    out = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
    ref = [d.clone() for d, _ in sets]
    lookups = {v: (d_bm if v in (0, 5, 11) else table) for v in names}
    bad = []
    for v in names:
        for i, (d, p) in enumerate(sets):
            assert xec.erase(d, p, S, bs, k, m, d_bm, s) == 0
            assert L.lab_decode(v, d.data_ptr(), p.data_ptr(), lookups[v].data_ptr(), out.data_ptr(),
                                S, bs, k, m, sh) == 0
            torch.cuda.synchronize()
            if v not in (3, 7, 8, 12, 14, 15, 16, 17) and not torch.equal(d, ref[i]):
                bad.append(names[v])
            d.copy_(ref[i])
    for (d, p), r in zip(sets, ref):  # d12 writes into the other set, d17 into parity
        d.copy_(r)
        assert xec.encode(d, p, S, bs, k, m, s) == 0
    print("incorrect decode variants:", bad, flush=True)
    b_dec = S * (k // m + 1) * bs

    def run(fn):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.iters)]
        fn(0)
        for i in range(args.iters):
            ev[2 * i].record(s)
            fn(i + 1)
            ev[2 * i + 1].record(s)
        torch.cuda.synchronize()
        return [ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(args.iters)]

    res = {n: [] for n in names.values()}
    res["product_decode"] = []
    res["product_encode"] = []
    for _ in range(args.rounds):
        res["product_encode"] += run(lambda i: xec.encode(sets[i % 2][0], sets[i % 2][1], S, bs, k, m, s))
        res["product_decode"] += run(lambda i: xec.decode(sets[i % 2][0], sets[i % 2][1], S, bs, k, m,
                                                          h_bm, d_bm, s))
        for v, n in names.items():
            # d12: the rebuilt block goes to the same offset of the OTHER set's data buffer
            outp = (lambda i: sets[(i + 1) % 2][0].data_ptr()) if v == 12 else (lambda i: out.data_ptr())
            res[n] += run(lambda i, v=v, outp=outp: L.lab_decode(
                v, sets[i % 2][0].data_ptr(), sets[i % 2][1].data_ptr(), lookups[v].data_ptr(), outp(i),
                S, bs, k, m, sh))
    for n, ts in sorted(res.items(), key=lambda kv: statistics.median(kv[1])):
        med = statistics.median(ts)
        b = S * (k + m) * bs if n == "product_encode" else b_dec
        print(f"{n:24s} ms_med {med:.4f}  GBps_med {b / (med * 1e-3) / 1e9:.1f}")



def wburst_lab(args, L, torch, sets, S, k, bs, s, sh):
    """Overwrites the data buffers (4 GiB each at the default shape, far past
    the Infinity Cache); nothing else runs in this mode."""
    L.lab_wburst.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    L.lab_set_ceiling_lds.argtypes = [ctypes.c_uint32]
    names = ["1K_nt", "4K_nt", "16K_nt", "1K_sc1", "4K_sc1", "16K_sc1", "4K_by_256thr_nt",
             "1K_xcdgrp4_nt", "2K_nt", "8K_nt", "1K_xcdgrp4_sc1", "1K_xcdgrp2_nt"]
    occs = [int(x) for x in args.occ.split(",")]
    nbytes = S * k * bs

    def run(fn):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.iters)]
        fn(0)
        for i in range(args.iters):
            ev[2 * i].record(s)
            fn(i + 1)
            ev[2 * i + 1].record(s)
        torch.cuda.synchronize()
        return [ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(args.iters)]

    res = {f"{n}_o{w}": [] for w in occs for n in names}
    for _ in range(args.rounds):
        for w in occs:
            L.lab_set_ceiling_lds(0 if w <= 0 or w >= 8 else ((160 * 1024) // (4 * w)) & ~511)
            for v, n in enumerate(names):
                res[f"{n}_o{w}"] += run(lambda i, v=v: L.lab_wburst(
                    v, sets[i % 2][0].data_ptr(), nbytes, sh))
    L.lab_set_ceiling_lds(0)
    out = {}
    for n, ts in res.items():
        med = statistics.median(ts)
        out[n] = {"ms_med": round(med, 4), "GBps_med": round(nbytes / (med * 1e-3) / 1e9, 1)}
        print(f"{n:16s} {out[n]}", flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps({"bytes": nbytes, "results": out}, indent=1))


def wscatter_lab(args, L, torch, sets, S, k, bs, s, sh):
    """Write-only streams of up to 1 GiB into the data buffers: dense, and as the
    decode's rebuilt blocks land -- one block per stripe (config 3: 1 MiB per
    16 MiB; 16+8 x 64 KiB: 64 KiB per 1.5 MiB; config 4: 4 KiB per 132 KiB),
    each as one-wave 1 KiB stores; nt and sc1.  Overwrites the data buffers."""
    L.lab_wscatter.argtypes = [ctypes.c_int, ctypes.c_void_p] + [ctypes.c_uint64] * 3 + [ctypes.c_void_p]
    total = 1 << 30
    span = S * k * bs
    shapes = {"dense_1M": (1 << 20, 1 << 20), "cfg3_1M_per_16M": (1 << 20, 16 << 20),
              "m8_64K_per_1.5M": (64 << 10, 1536 << 10), "cfg4_4K_per_132K": (4 << 10, 132 << 10),
              "4K_per_16K": (4 << 10, 16 << 10), "64K_per_128K": (64 << 10, 128 << 10)}
    cases = []
    for name, (blk, stride) in shapes.items():
        nblk = total // blk
        if (nblk - 1) * stride + blk > span:
            nblk = (span - blk) // stride + 1
        for sc1 in (0, 1):
            cases.append((f"{name}_{'sc1' if sc1 else 'nt'}", sc1, blk, stride, nblk))

    def run(fn):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.iters)]
        fn(0)
        for i in range(args.iters):
            ev[2 * i].record(s)
            fn(i + 1)
            ev[2 * i + 1].record(s)
        torch.cuda.synchronize()
        return [ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(args.iters)]

    res = {c[0]: [] for c in cases}
    for _ in range(args.rounds):
        for name, sc1, blk, stride, nblk in cases:
            res[name] += run(lambda i, a=(sc1, blk, stride, nblk): L.lab_wscatter(
                a[0], sets[i % 2][0].data_ptr(), a[1], a[2], a[3], sh))
    out = {}
    for name, sc1, blk, stride, nblk in cases:
        med = statistics.median(res[name])
        out[name] = {"block": blk, "stride": stride, "blocks": nblk, "bytes": nblk * blk,
                     "ms_med": round(med, 4), "GBps_med": round(nblk * blk / (med * 1e-3) / 1e9, 1)}
        print(f"{name:24s} {out[name]}", flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1))


def ceiling_lab(args, L, torch, xec, sets, S, k, m, bs, s, sh):
    L.lab_ceiling.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_uint64] * 4 + [ctypes.c_void_p]

    def run(fn):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * args.iters)]
        fn(0)
        for i in range(args.iters):
            ev[2 * i].record(s)
            fn(i + 1)
            ev[2 * i + 1].record(s)
        torch.cuda.synchronize()
        return [ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(args.iters)]

    L.lab_set_ceiling_lds.argtypes = [ctypes.c_uint32]
    occs = [int(x) for x in args.occ.split(",")]

    def lds(w):  # as csrc/xec_api.cpp lds_for_occupancy for one-wave workgroups
        return 0 if w <= 0 or w >= 8 else ((160 * 1024) // (4 * w)) & ~511

    base = {"read_only_16way": S * k * bs, "write_only": S * bs, "copy": 2 * S * bs,
            "read_only_16way_wg256": S * k * bs, "read_only_16way_wg128": S * k * bs}
    bytes_, res = {}, {}
    for w in occs:
        for n, b in base.items():
            bytes_[f"{n}_o{w}"] = b
        bytes_[f"product_encode_occ{w}"] = S * (k + m) * bs
    res = {n: [] for n in bytes_}
    for _ in range(args.rounds):
        for w in occs:
            assert xec.set_occupancy(w) == 0
            res[f"product_encode_occ{w}"] += run(
                lambda i: xec.encode(sets[i % 2][0], sets[i % 2][1], S, bs, k, m, s))
            L.lab_set_ceiling_lds(lds(w))
            for mode, n in enumerate(base):
                res[f"{n}_o{w}"] += run(lambda i, mode=mode: L.lab_ceiling(
                    mode, sets[i % 2][0].data_ptr(), sets[i % 2][1].data_ptr(), S, bs, k, m, sh))
    xec.set_occupancy(0)
    L.lab_set_ceiling_lds(0)
    out = {}
    for n, ts in res.items():
        med = statistics.median(ts)
        out[n] = {"ms_med": round(med, 4), "GBps_med": round(bytes_[n] / (med * 1e-3) / 1e9, 1),
                  "GBps_best": round(bytes_[n] / (min(ts) * 1e-3) / 1e9, 1)}
        print(f"{n:28s} {out[n]}", flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps({"shape": [S, k, m, bs], "results": out}, indent=1))


if __name__ == "__main__":
    main()
