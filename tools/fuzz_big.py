#!/usr/bin/env python3
"""Randomised round trips at real batch sizes (GPU box): the size-independent
property check of tests/test_gpu_fuzz.py, without the CPU oracle, so batches of
128 MiB - 2 GiB fit.  Per case: a random k, m (k % m == 0), block size and
stripe count; fill; encode, parity checked against a torch XOR of each class;
then a random loss pattern -- uniform (every stripe loses 1..m data blocks in
distinct classes), sparse (one stripe in ~9), skewed (a few stripes lose up to
m, the rest nothing), with lost parity blocks, or one failed device (the same
data block gone from every stripe: the automatic decode rotation's case) --
erased and rebuilt through every decode entry point and forced tiling, under a
per-case column rotation (xec_set_rotation: automatic, none or explicit).  A recoverable batch must come back
bit-exact with parity untouched; one with an unrecoverable stripe must be left
as erased (xec_decode_per_stripe: failing stripes only).

    python tools/fuzz_big.py [--cases 60] [--seed 1] [--out f.json]
    python tools/fuzz_big.py --pipeline ...   # the host-in/host-out pipeline instead

--pipeline: the batch lives in host memory (32-512 MiB; pinned, pageable, or
pageable data with pinned parity, case by case); xec_pipeline
encode must give the device encode's parity, and decode must restore the
erased host batch (only classes that lost a data block travel at >= 64 KiB
blocks, csrc/xec_pipeline.cpp), or leave it untouched when a stripe is
unrecoverable.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))

PATHS = ["auto", "stripe", "class", "list", "mask", "per_stripe", "device", "device_list"]


def loss_pattern(np, rng, S, k, m, kind):
    """Bitmap (S, k+m) uint8, 0 = lost."""
    bm = np.ones((S, k + m), np.uint8)
    nm = k // m
    if kind == "device":  # one failed device: the same data block in every stripe
        bm[:, int(rng.integers(0, k))] = 0
        return bm
    if kind == "uniform":
        nlost = rng.integers(1, m + 1, size=S)
    elif kind == "sparse":
        nlost = np.where(rng.random(S) < 1 / 9, rng.integers(1, m + 1, size=S), 0)
    else:  # skewed / parity
        nlost = np.where(rng.random(S) < 0.05, m, 0) if kind == "skewed" else \
            rng.integers(0, m + 1, size=S)
    order = np.argsort(rng.random((S, m)), axis=1)  # distinct classes per stripe
    rows = np.arange(S)
    for q in range(m):
        sel = nlost > q
        cls = order[:, q]
        mem = rng.integers(0, nm, size=S)
        bm[rows[sel], (cls + m * mem)[sel]] = 0
    if kind == "parity":  # lose the parity of classes that lost no data block
        data_lost_cls = np.zeros((S, m), bool)
        for j in range(m):
            data_lost_cls[:, j] = (bm[:, j:k:m] == 0).any(axis=1)
        drop = (~data_lost_cls) & (rng.random((S, m)) < 0.3)
        bm[:, k:][drop] = 0
    return bm


def recoverable(np, bm, k, m):
    lost = bm == 0
    ok = np.ones(bm.shape[0], bool)
    for j in range(m):
        ok &= (lost[:, j:k:m].sum(axis=1) + lost[:, k + j]) <= 1
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=60)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--pipeline", action="store_true")
    ap.add_argument("--start", type=int, default=0,
                    help="--pipeline: draw but skip the cases before this one (re-run one case "
                         "of a seed's sequence)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import numpy as np
    import torch

    import xec

    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    s = torch.cuda.current_stream()
    rng = np.random.default_rng(args.seed)
    if args.pipeline:
        return pipeline_fuzz(args, np, torch, xec, s, rng)
    log = []
    t_start = time.time()
    for case in range(args.cases):
        m = int(rng.choice([1, 1, 2, 4, 8, 3, 5]))
        k = m * int(rng.integers(1, max(2, 64 // m) + 1))
        bs = 256 * int(rng.choice([1, 3, 16, 64, 256, 1024, 4096]))
        target = int(rng.integers(128 << 20, 2 << 30))
        S = max(1, target // (k * bs))
        kind = ["uniform", "sparse", "skewed", "parity", "device"][case % 5]
        unrec = case % 7 == 3  # one unrecoverable stripe
        rot = int(rng.choice([0, 0, -1, 1, 3, 129]))
        assert xec.set_rotation(rot) == 0
        d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
        p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
        assert xec.fill_splitmix64(d, S, k * bs, 5000 + case, s) == 0
        assert xec.encode(d, p, S, bs, k, m, s) == 0
        # parity == XOR over each class (as bench.py verifies)
        blocks = d.view(S, k // m, m, bs)
        red = blocks[:, 0].clone()
        for r in range(1, k // m):
            red.bitwise_xor_(blocks[:, r])
        enc_ok = bool(torch.equal(red.reshape(-1), p))
        del red, blocks
        orig_d = d.clone()
        orig_p = p.clone()
        bm = loss_pattern(np, rng, S, k, m, kind)
        if unrec:
            c = int(rng.integers(0, S))
            bm[c, :] = 1
            bm[c, 0] = 0
            bm[c, k] = 0
        rec = recoverable(np, bm, k, m)
        h_bm = torch.from_numpy(bm.reshape(-1).copy()).pin_memory()
        d_bm = h_bm.to("cuda")
        rec_t = torch.from_numpy(rec).to("cuda")
        results = {}
        for path in PATHS:
            d.copy_(orig_d)
            p.copy_(orig_p)
            assert xec.erase(d, p, S, bs, k, m, d_bm, s) == 0
            erased = d.clone()
            erased_p = p.clone()
            scratch = torch.empty_like(d_bm)
            if path in ("auto", "stripe", "class", "list", "mask"):
                xec.set_decode_tiling({"auto": 0, "stripe": 1, "class": 2, "list": 3, "mask": 4}[path])
                st = int(xec.decode(d, p, S, bs, k, m, h_bm, scratch, s))
                xec.set_decode_tiling(0)
            elif path == "per_stripe":
                st = int(xec.decode_per_stripe(d, p, S, bs, k, m, h_bm, scratch, None, s))
            else:
                dst = torch.full((1,), -1, dtype=torch.int32, device="cuda")
                if path == "device":
                    assert xec.decode_device(d, p, S, bs, k, m, d_bm, dst, s) == 0
                    torch.cuda.synchronize()
                    st = int(dst.item())
                else:
                    n = xec.device_list_bytes(S, k, m)
                    w = torch.empty((n + 3) // 4, dtype=torch.int32, device="cuda")
                    st = int(xec.decode_device_list(d, p, S, bs, k, m, d_bm, w, n, dst, s))
                    if st == 0:
                        torch.cuda.synchronize()
                        st = int(dst.item())
                    del w
            torch.cuda.synchronize()
            par_ok = bool(torch.equal(p, erased_p))
            if k > 256 and path in ("per_stripe", "device_list"):
                ok = st == 1 and bool(torch.equal(d, erased))
            elif path == "per_stripe":
                want = torch.where(rec_t[:, None], orig_d.view(S, -1), erased.view(S, -1))
                ok = st == (0 if rec.all() else 4) and bool(torch.equal(d.view(S, -1), want))
                del want
            elif rec.all():
                ok = st == 0 and bool(torch.equal(d, orig_d))
            else:
                ok = st == 4 and bool(torch.equal(d, erased))
            results[path] = bool(ok and par_ok)
            del erased, erased_p
        row = {"case": case, "k": k, "m": m, "bs": bs, "S": S, "GiB": round(S * k * bs / 2**30, 3),
               "pattern": kind, "rotation": rot, "lost_data_blocks": int((bm[:, :k] == 0).sum()),
               "recoverable": bool(rec.all()), "encode_ok": enc_ok, "decode_ok": results}
        log.append(row)
        bad = (not enc_ok) or not all(results.values())
        print(("FAIL " if bad else "ok   ") + json.dumps(row), flush=True)
        del d, p, orig_d, orig_p, d_bm, h_bm, rec_t
        torch.cuda.empty_cache()
        if bad:
            break
    n_ok = sum(1 for r in log if r["encode_ok"] and all(r["decode_ok"].values()))
    summary = {"cases": len(log), "all_ok": n_ok == len(log), "seconds": round(time.time() - t_start, 1)}
    print(json.dumps(summary), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps({"summary": summary, "cases": log}, indent=1))
    sys.exit(0 if summary["all_ok"] else 1)


def pipeline_fuzz(args, np, torch, xec, s, rng):
    log = []
    t_start = time.time()
    for case in range(args.cases):
        m = int(rng.choice([1, 1, 2, 4, 8, 3]))
        k = m * int(rng.integers(1, max(2, 32 // m) + 1))
        bs = 256 * int(rng.choice([1, 16, 64, 256, 1024, 4096]))
        target = int(rng.integers(32 << 20, 512 << 20))
        S = max(1, target // (k * bs))
        chunk = int(rng.integers(1, 17))
        ns = int(rng.integers(1, 5))
        kind = ["uniform", "sparse", "skewed", "parity"][case % 4]
        unrec = case % 7 == 3
        if case < args.start:  # advance the generator exactly as the case would
            loss_pattern(np, rng, S, k, m, kind)
            if unrec:
                rng.integers(0, S)
            continue
        d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
        p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
        assert xec.fill_splitmix64(d, S, k * bs, 9000 + case, s) == 0
        assert xec.encode(d, p, S, bs, k, m, s) == 0
        # host buffers pinned, pageable (file / socket buffers: the pipeline's
        # bounce-buffer path), or pageable data with pinned parity, in turn
        mem = ["pinned", "pageable", "mixed"][case % 3]
        h_d = torch.empty(S * k * bs, dtype=torch.uint8)
        h_p = torch.empty(S * m * bs, dtype=torch.uint8)
        if mem == "pinned":
            h_d = h_d.pin_memory()
        if mem != "pageable":
            h_p = h_p.pin_memory()
        h_d.copy_(d)
        ref_p = p.cpu()
        ref_d = h_d.clone()
        del d, p
        bm = loss_pattern(np, rng, S, k, m, kind)
        if unrec:
            c = int(rng.integers(0, S))
            bm[c, :] = 1
            bm[c, 0] = 0
            bm[c, k] = 0
        rec = recoverable(np, bm, k, m)
        h_bm = torch.from_numpy(bm.reshape(-1).copy()).pin_memory()
        with xec.Pipeline(chunk, bs, k, m, ns) as pl:
            h_p.zero_()
            enc_ok = pl.encode(h_d, h_p, S) == 0 and bool(torch.equal(h_p, ref_p))
            hv = h_d.numpy().reshape(S, k, bs)
            hv[bm[:, :k] == 0] = 0
            erased = h_d.clone()
            st = int(pl.decode(h_d, h_p, S, h_bm))
        if rec.all():
            dec_ok = st == 0 and bool(torch.equal(h_d, ref_d))
        else:
            dec_ok = st == 4 and bool(torch.equal(h_d, erased))
        if not dec_ok:  # where: which stripes / blocks, lost or not, zero or stale
            got = h_d.numpy().reshape(S, k, bs)
            want = (ref_d if rec.all() else erased).numpy().reshape(S, k, bs)
            bad = np.argwhere((got != want).any(axis=2))
            print("diagnose " + json.dumps({
                "status": st, "bad_blocks": int(len(bad)), "first_bad": bad[:12].tolist(),
                "bad_chunks": sorted(set((bad[:, 0] // chunk).tolist()))[:24],
                "bad_were_lost": int((bm[bad[:, 0], bad[:, 1]] == 0).sum()),
                "bad_zero": int(sum((got[c, i] == 0).all() for c, i in bad[:200])),
                "bad_eq_erased": int(sum((got[c, i] == erased.numpy().reshape(S, k, bs)[c, i]).all()
                                         for c, i in bad[:200])),
                "parity_intact": bool(torch.equal(h_p, ref_p)),
                "chunks_total": (S + chunk - 1) // chunk}), flush=True)
        row = {"case": case, "k": k, "m": m, "bs": bs, "S": S, "chunk": chunk, "streams": ns,
               "MiB": round(S * k * bs / 2**20, 1), "pattern": kind, "host_memory": mem,
               "recoverable": bool(rec.all()), "encode_ok": enc_ok, "decode_ok": dec_ok}
        log.append(row)
        bad = not (enc_ok and dec_ok)
        print(("FAIL " if bad else "ok   ") + json.dumps(row), flush=True)
        del h_d, h_p, ref_d, ref_p, erased, h_bm
        if bad:
            break
    n_ok = sum(1 for r in log if r["encode_ok"] and r["decode_ok"])
    summary = {"cases": len(log), "all_ok": n_ok == len(log), "seconds": round(time.time() - t_start, 1)}
    print(json.dumps(summary), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps({"summary": summary, "cases": log}, indent=1))
    sys.exit(0 if summary["all_ok"] else 1)


if __name__ == "__main__":
    main()
