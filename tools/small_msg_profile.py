#!/usr/bin/env python3
"""Kernel time against call time at the reference's own message size.

The reference's committed GPU sweep is 8 MiB messages (MESSAGE_SIZE,
/root/reference/src/benchmark/bm_config.hpp:51; rows 1118-1141 of
results/raw/final_results.csv, kept as data in tools/reference_gpu_rows.csv).
For each of those 24 rows this runs bin/xec_bench (the BM_generic-equivalent
loop over the XorecBenchmarkHip plugin) twice:

  * plain, all rows in one process: the per-call wall time the harness reports
    (encode_time_ns / decode_time_ns, the stream synchronise included);
  * one process per row under `rocprofv3 --kernel-trace --stats`: the average
    duration of the encode and decode kernels themselves.

The difference is what a call costs beyond its kernel: launch, kernel-argument
copy, the host scan, the synchronise.  `--lib DIR` puts DIR first on
LD_LIBRARY_PATH (xec_bench finds libxec_hip.so through RUNPATH), so two
builds of the library can be compared in one GPU call.

    python tools/small_msg_profile.py --out gpurun_out/x/small.json [--lib tools/ab/r5] [--tag r5]
"""
from __future__ import annotations

import argparse
import csv
import io
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
BENCH = ROOT / "erasure-code-benchmark_amd" / "bin" / "xec_bench"
ROWS = ROOT / "tools" / "reference_gpu_rows.csv"
MESSAGE = 8 << 20


def reference_rows():
    rows = [r for r in csv.DictReader(line for line in ROWS.open() if not line.startswith("#"))
            if int(r["message_size_B"]) == MESSAGE]
    out = []
    for r in rows:
        total, data = (int(x) for x in r["EC"].strip('"()').split("/"))
        out.append({"ref_line": int(r["line"]), "block_B": int(r["block_size_B"]), "k": data,
                    "m": total - data, "lost": int(r["lost_blocks"]), "EC": r["EC"].strip('"')})
    return out


def run_bench(cfgs, iters, warmup, env, prof_dir=None):
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as f:
        for c in cfgs:
            f.write(f"{MESSAGE} {c['block_B']} {c['k']} {c['m']} {c['lost']}\n")
        sweep = f.name
    cmd = [str(BENCH), "-g", "xorec-hip", "--sweep", sweep, "-i", str(iters), "-w", str(warmup),
           "--seed", "1896", "--stdout"]
    if prof_dir is not None:
        cmd = ["rocprofv3", "--kernel-trace", "--stats", "-d", str(prof_dir), "-o", "kt",
               "--output-format", "csv", "--"] + cmd
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    os.unlink(sweep)
    if p.returncode != 0:
        sys.exit(f"xec_bench failed rc={p.returncode}: {p.stderr[-3000:]}\n{p.stdout[-2000:]}")
    text = p.stdout[p.stdout.find("name,"):] if "name," in p.stdout else p.stdout
    return list(csv.DictReader(io.StringIO(text)))


def kernel_stats(prof_dir: Path):
    files = sorted(prof_dir.rglob("*kernel_stats.csv"))
    if not files:
        return {}
    out = {}
    for r in csv.DictReader(files[-1].open()):
        out[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                          "min_ns": float(r["MinNs"])}
    return out


def pick(stats, needle):
    hits = {n: v for n, v in stats.items() if needle in n}
    if not hits:
        return None, None
    name = max(hits, key=lambda n: hits[n]["calls"])
    return name, hits[name]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--lib", default="", help="directory with a libxec_hip.so to use instead")
    ap.add_argument("--tag", default="")
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--lines", default="", help="comma list of reference lines (default: all 24)")
    ap.add_argument("--no-prof", action="store_true", help="call times only, no rocprofv3 runs")
    args = ap.parse_args()
    env = dict(os.environ)
    if args.lib:
        env["LD_LIBRARY_PATH"] = str(Path(args.lib).resolve()) + (
            ":" + env["LD_LIBRARY_PATH"] if env.get("LD_LIBRARY_PATH") else "")
    out_path = Path(args.out)
    out_path.parent.mkdir(parents=True, exist_ok=True)
    cfgs = reference_rows()
    if args.lines:
        keep = {int(x) for x in args.lines.split(",")}
        cfgs = [c for c in cfgs if c["ref_line"] in keep]
    plain = run_bench(cfgs, args.iters, args.warmup, env)
    assert len(plain) == len(cfgs), (len(plain), len(cfgs))
    rows = []
    for c, o in zip(cfgs, plain):
        pdir = out_path.parent / f"prof_{args.tag or 'wt'}_{c['ref_line']}"
        if not args.no_prof:
            run_bench([c], args.iters, args.warmup, env, prof_dir=pdir)
        st = {} if args.no_prof else kernel_stats(pdir)
        en, ev = pick(st, "encode_kernel")
        dn, dv = pick(st, "decode_")
        S = MESSAGE // (c["k"] * c["block_B"])
        enc_bytes = S * (c["k"] + c["m"]) * c["block_B"]
        row = dict(c, stripes=S, err=o.get("err_msg", ""),
                   enc_call_us=round(float(o["encode_time_ns"]) / 1e3, 2),
                   dec_call_us=round(float(o["decode_time_ns"]) / 1e3, 2),
                   enc_kernel=en, enc_kernel_ns=round(ev["avg_ns"]) if ev else None,
                   enc_kernel_calls=ev["calls"] if ev else 0,
                   dec_kernel=dn, dec_kernel_ns=round(dv["avg_ns"]) if dv else None,
                   dec_kernel_calls=dv["calls"] if dv else 0)
        if ev:
            row["enc_kernel_TBps"] = round(enc_bytes / ev["avg_ns"] / 1e3, 3)
            row["enc_overhead_us"] = round(row["enc_call_us"] - ev["avg_ns"] / 1e3, 2)
        if dv:
            row["dec_overhead_us"] = round(row["dec_call_us"] - dv["avg_ns"] / 1e3, 2)
        rows.append(row)
        print(f"{c['ref_line']} {c['block_B'] >> 10:2d}KiB {c['EC']:>7s} lost={c['lost']} "
              f"enc call {row['enc_call_us']:7.2f} us kernel {row['enc_kernel_ns']} ns "
              f"({row.get('enc_kernel_TBps')} TB/s)  dec call {row['dec_call_us']:7.2f} us "
              f"kernel {row['dec_kernel_ns']} ns", flush=True)
    out_path.write_text(json.dumps({"tag": args.tag, "lib": args.lib or "in-tree",
                                    "iterations": args.iters, "warmup": args.warmup,
                                    "message_B": MESSAGE, "rows": rows}, indent=1) + "\n")


if __name__ == "__main__":
    main()
