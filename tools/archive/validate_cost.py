#!/usr/bin/env python3
"""What the device-side validation payload costs next to one encode
(VERDICT r1 item 7): xec_write_validation_pattern and xec_validate_blocks
(the GPU check_for_corruption of the plugin harness, abstract_bm.cpp:41-50 /
xorec_gpu_cmp_bm.cpp:91-104) over a workload's data blocks, with the lane-per-
block and the wave-per-block kernels, against xec_encode of the same batch.
HIP events on torch's current stream, median of N launches.

Validation must read every data byte once (S*k*bs), so its floor is the HBM
read time of the data -- about the encode's own time, which reads the same
bytes and writes 1/k more.

    python tools/archive/validate_cost.py [--workload cfg3] [--iters 10] [--out f.json]
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

from bench import workload_shape  # noqa: E402


def timed(fn, iters, stream):
    import torch
    ms = []
    for _ in range(iters):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(stream)
        assert fn() == 0
        b.record(stream)
        b.synchronize()
        ms.append(a.elapsed_time(b))
    return statistics.median(ms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    import xec

    k, m, bs, S, _ = workload_shape(a.workload)
    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    s = torch.cuda.current_stream()
    n = S * k
    d = torch.empty(n * bs, dtype=torch.uint8, device="cuda")
    p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")
    res = {"workload": a.workload, "k": k, "m": m, "bs": bs, "S": S, "data_blocks": n,
           "data_bytes": n * bs, "iters": a.iters}
    enc = timed(lambda: xec.encode(d, p, S, bs, k, m, s), a.iters, s)
    res["encode_ms"] = round(enc, 4)
    for mode, name in ((1, "lane_per_block"), (2, "wave_per_block"), (0, "auto")):
        assert xec.set_validate_kernel(mode) == 0
        w = timed(lambda: xec.write_validation_pattern(d, n, bs, 5, s), max(2, a.iters // 3), s)
        v = timed(lambda: xec.validate_blocks(d, n, bs, bad, s), a.iters, s)
        torch.cuda.synchronize()
        assert int(bad.item()) == 0, (name, int(bad.item()))
        res[name] = {"pattern_ms": round(w, 4), "validate_ms": round(v, 4),
                     "validate_GBps": round(n * bs / v / 1e6, 1),
                     "validate_over_encode": round(v / enc, 3)}
        print(name, res[name], flush=True)
    xec.set_validate_kernel(0)
    line = json.dumps(res)
    print(line)
    if a.out:
        Path(a.out).write_text(line + "\n")


if __name__ == "__main__":
    main()
