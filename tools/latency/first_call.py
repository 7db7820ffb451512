#!/usr/bin/env python3
"""Cold-start cost of the C ABI in a fresh process: xec_init, then the first
and the second call of each kind on a tiny batch (k=4+1, 4 KiB, 8 stripes),
each followed by a stream synchronise.  A service pays the first call once;
the reference pays its equivalent inside xorec_gpu_init / the first launch
(xorec_gpu_cmp.cu:7-27).

    python tools/latency/first_call.py [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    t0 = time.perf_counter()
    import torch
    t_torch = time.perf_counter() - t0
    import xec
    torch.cuda.set_device(0)
    s = torch.cuda.current_stream()
    S, k, m, bs = 8, 4, 1, 4096
    d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
    p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
    import numpy as np
    bm = np.ones((S, k + m), np.uint8)
    bm[:, 1] = 0
    h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
    d_bm = h_bm.to("cuda")
    torch.cuda.synchronize()

    def timed(fn):
        t = time.perf_counter()
        rc = fn()
        s.synchronize()
        return round((time.perf_counter() - t) * 1e6, 1), int(rc)

    out = {"import_torch_s": round(t_torch, 2)}
    out["xec_init_us"] = timed(lambda: xec.init(0))
    for name, fn in (("fill", lambda: xec.fill_splitmix64(d, S, k * bs, 1, s)),
                     ("encode", lambda: xec.encode(d, p, S, bs, k, m, s)),
                     ("erase", lambda: xec.erase(d, p, S, bs, k, m, d_bm, s)),
                     ("decode", lambda: xec.decode(d, p, S, bs, k, m, h_bm, d_bm, s))):
        out[f"{name}_first_us"] = timed(fn)
        out[f"{name}_second_us"] = timed(fn)
    print(json.dumps(out), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
