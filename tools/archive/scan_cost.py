#!/usr/bin/env python3
"""What the host recoverability scan of xec_decode costs in the synchronous,
reference-shaped plugin path.

1. xec_check_bitmap (the same scan xec_decode runs, host only) timed on the
   bitmap of a workload (default cfg4: 65,536 stripes x 33 bytes, one lost
   data block per stripe), median of N calls;
2. bin/xec_bench (XorecBenchmarkHip in the BM_generic loop: every call ends in
   a stream synchronise, so nothing overlaps the scan) at the same shape:
   decode wall time per call;
3. the decode kernel alone (HIP events around xec_decode launched back to back
   on one stream, so each call's scan overlaps the previous kernel).

    python tools/archive/scan_cost.py [--workload cfg4] [--out f.json]
"""
from __future__ import annotations

import argparse
import csv
import io
import json
import statistics
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))

from bench import erasure_pattern, workload_shape  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg4")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import numpy as np
    import torch

    import xec

    k, m, bs, S, _ = workload_shape(a.workload)
    bm = np.ascontiguousarray(erasure_pattern(np, S, k, m).reshape(-1))
    ts = []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        st, needs = xec.check_bitmap(bm, S, k, m)
        ts.append(time.perf_counter() - t0)
        assert st == 0 and needs
    scan_us = statistics.median(ts) * 1e6

    # 3. device decode back to back
    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    stream = torch.cuda.current_stream()
    d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
    p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
    assert xec.fill_splitmix64(d, S, k * bs, 1, stream) == 0
    assert xec.encode(d, p, S, bs, k, m, stream) == 0
    h_bm = torch.from_numpy(bm).pin_memory()
    scratch = torch.empty(S * (k + m), dtype=torch.uint8, device="cuda")
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(a.iters)]
    for i in range(a.iters):
        evs[i][0].record(stream)
        assert xec.decode(d, p, S, bs, k, m, h_bm, scratch, stream) == 0
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    kern_us = statistics.median(x.elapsed_time(y) for x, y in evs[2:]) * 1e3
    # the same call, synchronised each time (what the plugin does), wall clock
    ws = []
    for _ in range(a.iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        assert xec.decode(d, p, S, bs, k, m, h_bm, scratch, stream) == 0
        torch.cuda.synchronize()
        ws.append(time.perf_counter() - t0)
    sync_us = statistics.median(ws[2:]) * 1e6
    del d, p
    torch.cuda.empty_cache()

    # 2. the plugin harness
    bench = ROOT / "erasure-code-benchmark_amd" / "bin" / "xec_bench"
    r = subprocess.run([str(bench), "-g", "xorec-hip", "--stdout", "--message", str(S * k * bs),
                        "--block", str(bs), "--data", str(k), "--parity", str(m), "--lost", "1",
                        "-i", str(a.iters), "-w", "3", "--seed", "5"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    row = next(csv.DictReader(io.StringIO(r.stdout)))
    plugin_us = float(row["decode_time_ns"]) / 1e3
    out = {"workload": a.workload, "k": k, "m": m, "bs": bs, "S": S,
           "host_scan_us_median": round(scan_us, 1),
           "decode_kernel_us_events": round(kern_us, 1),
           "decode_call_plus_sync_us_wall": round(sync_us, 1),
           "plugin_decode_us_mean": round(plugin_us, 1),
           "plugin_err": row["err_msg"],
           "scan_share_of_plugin_decode": round(scan_us / plugin_us, 4),
           "plugin_over_kernel": round(plugin_us / kern_us, 4)}
    print(json.dumps(out), flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
