#!/usr/bin/env python3
"""xec_decode_device_list's launch grid (DESIGN.md §8 Next #3: on dense batches
it ran 9-19 % behind xec_decode_device's one workgroup per tile).

The device-list decode cannot see how many blocks its check kernel listed, so
it launches a fixed grid of what the chip holds at once and walks the list in
grid strides.  The alternative is a grid of one workgroup per POSSIBLE tile
(S*m entries x chunks) in which the workgroups past the list's end return at
once -- xec_set_launch's max_grid gives it without a rebuild.  Times, per
shape and loss density, in one process and interleaved rounds (HIP events
around each call, the check kernel included):

  device       xec_decode_device (stripe tiles over every stripe)
  list         xec_decode_device_list, default grid (persistent walk)
  list_full    xec_decode_device_list, one workgroup per possible tile

Every variant's rebuilt data is compared with the first's.

    python tools/lab/devlist_grid.py [--rounds 5] [--iters 10]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default="")
    ap.add_argument("--grids", default="",
                    help="comma list of extra xec_set_launch max_grid values for the list "
                         "decode (variants list_g<N>)")
    args = ap.parse_args()
    grids = [int(x) for x in args.grids.split(",") if x]
    import numpy as np
    import torch

    import xec
    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    s = torch.cuda.current_stream()
    shapes = [("cfg3", 16, 1, 1 << 20, 256), ("cfg4", 32, 1, 4096, 65536),
              ("cfg2", 8, 1, 65536, 1024), ("16+8x64K", 16, 8, 65536, 16384)]
    out = []
    for name, k, m, bs, S in shapes:
        d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
        p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
        assert xec.fill_splitmix64(d, S, k * bs, 1896, s) == 0
        assert xec.encode(d, p, S, bs, k, m, s) == 0
        work = torch.empty(xec.device_list_bytes(S, k, m), dtype=torch.uint8, device="cuda")
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        for density in ("every", "1in9"):
            bm = np.ones((S, k + m), np.uint8)
            rows = np.arange(S) if density == "every" else np.arange(4, S, 9)
            bm[rows, (7 * rows) % k] = 0
            d_bm = torch.from_numpy(bm.reshape(-1)).to("cuda")
            lost = len(rows)

            variants = ["device", "list", "list_full"] + [f"list_g{g}" for g in grids]

            def run(variant):
                if variant == "device":
                    return xec.decode_device(d, p, S, bs, k, m, d_bm, status, s)
                mg = ((1 << 31) - 1 if variant == "list_full" else
                      int(variant[6:]) if variant.startswith("list_g") else 0)
                assert xec.set_launch(0, mg, 0, 0) == 0
                try:
                    return xec.decode_device_list(d, p, S, bs, k, m, d_bm, work, work.numel(),
                                                  status, s)
                finally:
                    xec.set_launch(0, 0, 0, 0)

            ref = None
            for v in variants:  # the same bytes from every variant
                assert xec.erase(d, p, S, bs, k, m, d_bm, s) == 0
                assert run(v) == 0
                torch.cuda.synchronize()
                assert int(status.item()) == 0
                got = d.clone()
                ref = got if ref is None else ref
                assert torch.equal(got, ref), (name, density, v)
            del ref, got
            times = {v: [] for v in variants}
            for _ in range(args.rounds):
                for v in times:
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.iters + 1)]
                    ev[0].record(s)
                    for i in range(args.iters):
                        assert run(v) == 0
                        ev[i + 1].record(s)
                    torch.cuda.synchronize()
                    times[v] += [ev[i].elapsed_time(ev[i + 1]) for i in range(args.iters)]
            b = lost * (k // m + 1) * bs
            row = {"shape": name, "k": k, "m": m, "bs": bs, "S": S, "density": density,
                   "lost_blocks": lost}
            for v, t in times.items():
                ms = statistics.median(t)
                row[v] = {"ms": round(ms, 4), "GBps": round(b / ms / 1e6, 1)}
            row["list_full_over_list"] = round(row["list"]["ms"] / row["list_full"]["ms"], 3)
            row["list_full_over_device"] = round(row["device"]["ms"] / row["list_full"]["ms"], 3)
            print(json.dumps(row), flush=True)
            out.append(row)
        del d, p, work
        torch.cuda.empty_cache()
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
