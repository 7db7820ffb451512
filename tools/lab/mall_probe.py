#!/usr/bin/env python3
"""Is bench.py's decode helped by the 256 MiB Infinity Cache (MALL)?

Times the product decode of a buffer set in three situations, interleaved:
  rotation -- bench.py's own order (encode set s%3, then decode set (s+2)%3);
  flushed  -- the same decode right after 2 GiB of plain stores + a 2 GiB read of a
              scratch buffer (whatever the MALL held of the set is gone);
  hot      -- the decode right after the encode of the SAME set (its parity was
              just written: the most the MALL could give).
If rotation ~= flushed, the bench's decode number carries no cache credit.

    python tools/lab/mall_probe.py [--workload cfg2] [--rounds 5]
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

from bench import algorithmic_bytes, erasure_pattern, workload_shape  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import numpy as np
    import torch

    import xec

    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    k, m, bs, S, _ = workload_shape(args.workload)
    s = torch.cuda.current_stream()
    sets = []
    for i in range(3):
        d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
        p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
        assert xec.fill_splitmix64(d, S, k * bs, 1896 + 7919 * i, s) == 0
        assert xec.encode(d, p, S, bs, k, m, s) == 0
        sets.append((d, p))
    h_bm = torch.from_numpy(erasure_pattern(np, S, k, m).reshape(-1)).pin_memory()
    scratch = [h_bm.to("cuda") for _ in range(3)]
    flush_buf = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")
    b_enc, b_dec = algorithmic_bytes(S, k, m, bs)

    def enc(i):
        assert xec.encode(sets[i][0], sets[i][1], S, bs, k, m, s) == 0

    def dec(i, evs):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        assert xec.decode(sets[i][0], sets[i][1], S, bs, k, m, h_bm, scratch[i], s) == 0
        e1.record(s)
        evs.append((e0, e1))

    def flush():
        flush_buf.fill_(7)
        flush_buf.view(torch.int64).sum()

    res = {"rotation": [], "flushed": [], "hot": []}
    for _ in range(args.rounds):
        for name in res:
            evs = []
            for it in range(args.iters * 3):
                if name == "rotation":
                    enc(it % 3)
                    dec((it + 2) % 3, evs)
                elif name == "flushed":
                    enc(it % 3)
                    flush()
                    dec((it + 2) % 3, evs)
                else:
                    enc(it % 3)
                    dec(it % 3, evs)
            torch.cuda.synchronize()
            res[name] += [a.elapsed_time(b) for a, b in evs[3:]]
    out = {"workload": args.workload, "results": {}}
    for n, ts in res.items():
        med = statistics.median(ts)
        out["results"][n] = {"dec_ms_med": round(med, 4), "dec_GBps": round(b_dec / med / 1e6, 1)}
        print(n, out["results"][n], flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
