#!/usr/bin/env python3
"""Sustained-load check on one MI355X: for --seconds, every step encodes one of
two resident config-3 batches, erases a fresh random recoverable pattern (one
lost data block per stripe, a new draw each step), rebuilds it with
xec_decode_device (bitmap in HBM) or xec_decode (host bitmap) alternately, and
compares parity and data with the batch's pristine copy on the device.  Any
mismatch stops the run.  Prints a progress line every ~10 s.

    python tools/soak.py [--seconds 180] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180.0)
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import numpy as np
    import torch

    import xec

    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    s = torch.cuda.current_stream()
    k, m, bs, S = 16, 1, 1 << 20, 256
    sets = []
    for i in range(2):
        d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
        p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
        assert xec.fill_splitmix64(d, S, k * bs, 4000 + 97 * i, s) == 0
        assert xec.encode(d, p, S, bs, k, m, s) == 0
        sets.append((d, p, d.clone(), p.clone()))
    rng = np.random.default_rng(11)
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    t0 = time.time()
    last = t0
    steps = bad = 0
    while time.time() - t0 < args.seconds:
        d, p, d0, p0 = sets[steps % 2]
        assert xec.encode(d, p, S, bs, k, m, s) == 0
        bm = np.ones((S, k + m), np.uint8)
        bm[np.arange(S), rng.integers(0, k, size=S)] = 0
        h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
        d_bm = h_bm.to("cuda", non_blocking=True)
        assert xec.erase(d, p, S, bs, k, m, d_bm, s) == 0
        if steps % 2:
            assert xec.decode_device(d, p, S, bs, k, m, d_bm, st, s) == 0
        else:
            assert xec.decode(d, p, S, bs, k, m, h_bm, torch.empty_like(d_bm), s) == 0
        ok = bool(torch.equal(d, d0)) and bool(torch.equal(p, p0))
        if steps % 2:
            ok &= int(st.item()) == 0
        steps += 1
        if not ok:
            bad += 1
            break
        if time.time() - last > 10:
            last = time.time()
            print(f"t={last - t0:.0f}s steps={steps} mismatches={bad}", flush=True)
    torch.cuda.synchronize()
    out = {"seconds": round(time.time() - t0, 1), "steps": steps, "mismatches": bad,
           "shape": f"k={k}+{m}, {bs >> 20} MiB x {S} stripes", "ok": bad == 0}
    print(json.dumps(out), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1))
    sys.exit(0 if bad == 0 else 1)


if __name__ == "__main__":
    main()
