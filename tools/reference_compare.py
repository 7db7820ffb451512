#!/usr/bin/env python3
"""Re-run the reference's own published GPU benchmark rows on MI355X.

tools/reference_gpu_rows.csv holds the 53 "XOR-EC (GPU Computation)" rows of
the reference's results/raw/final_results.csv (Tesla V100; data only).  Every
row's configuration (message size, block size, EC (total/data), lost blocks)
is run through bin/xec_bench -- the XorecBenchmarkHip plugin under the
BM_generic-equivalent harness, same timing boundaries (wall clock around each
encode()/decode() call including the stream synchronise) and the same unit
(Gbit/s of message bytes) -- and compared row by row.

    python tools/reference_compare.py [--iters 100] [--warmup 20] [--out f.json]
"""
from __future__ import annotations

import argparse
import csv
import io
import json
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
BENCH = ROOT / "erasure-code-benchmark_amd" / "bin" / "xec_bench"
ROWS = Path(__file__).resolve().parent / "reference_gpu_rows.csv"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--out", default="")
    ap.add_argument("--csv-out", default="")
    args = ap.parse_args()

    ref = [r for r in csv.DictReader(line for line in ROWS.open() if not line.startswith("#"))]
    cfgs = []
    for r in ref:
        total, data = (int(x) for x in r["EC"].strip('"()').split("/"))
        cfgs.append((int(r["message_size_B"]), int(r["block_size_B"]), data, total - data,
                     int(r["lost_blocks"])))
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
        for c in cfgs:
            f.write(" ".join(map(str, c)) + "\n")
        sweep = f.name
    p = subprocess.run([str(BENCH), "-g", "xorec-hip", "--sweep", sweep, "-i", str(args.iters),
                        "-w", str(args.warmup), "--seed", "1896", "--stdout"],
                       capture_output=True, text=True, timeout=1500)
    if p.returncode != 0:
        sys.exit(f"xec_bench failed rc={p.returncode}: {p.stderr}\n{p.stdout[-2000:]}")
    if args.csv_out:
        Path(args.csv_out).write_text(p.stdout)
    ours = list(csv.DictReader(io.StringIO(p.stdout)))
    assert len(ours) == len(ref)
    rows = []
    for r, o in zip(ref, ours):
        row = {"ref_line": int(r["line"]), "message_B": int(r["message_size_B"]),
               "block_B": int(r["block_size_B"]), "EC": r["EC"].strip('"'),
               "lost": int(r["lost_blocks"]), "err": o["err_msg"],
               "enc_ref_Gbps": float(r["encode_throughput_Gbps"]),
               "enc_ours_Gbps": round(float(o["encode_throughput_Gbps"]), 1),
               "dec_ref_Gbps": float(r["decode_throughput_Gbps"]),
               "dec_ours_Gbps": round(float(o["decode_throughput_Gbps"]), 1)}
        row["enc_speedup"] = round(row["enc_ours_Gbps"] / row["enc_ref_Gbps"], 2)
        row["dec_speedup"] = round(row["dec_ours_Gbps"] / row["dec_ref_Gbps"], 2)
        rows.append(row)
        print(f"{row['ref_line']:5d} {row['message_B']>>20:4d}MiB {row['block_B']>>10:3d}KiB "
              f"{row['EC']:>7s} lost={row['lost']} enc {row['enc_ours_Gbps']:9.1f} vs "
              f"{row['enc_ref_Gbps']:8.1f} ({row['enc_speedup']:5.2f}x)  dec {row['dec_ours_Gbps']:9.1f}"
              f" vs {row['dec_ref_Gbps']:8.1f} ({row['dec_speedup']:5.2f}x) {row['err']}", flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps({"iterations": args.iters, "warmup": args.warmup,
                                              "rows": rows}, indent=1) + "\n")


if __name__ == "__main__":
    main()
