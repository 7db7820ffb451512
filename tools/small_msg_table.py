#!/usr/bin/env python3
"""Table of the reference's 8 MiB rows from tools/small_msg_profile.py runs.

    python tools/small_msg_table.py OUT.md BASE_a.json,BASE_b.json NEW_a.json,NEW_b.json

Each list holds runs of one library (alternated with the other's on one box);
every figure is the mean over its runs.  Columns: the encode call (wall clock
around encode() + stream synchronise, BM_generic's boundary) against the
encode kernel's rocprofv3 average duration and algorithmic rate, and the same
for decode, base -> new library.
"""
from __future__ import annotations

import json
import statistics
import sys
from pathlib import Path


def load(spec):
    return [json.loads(Path(f).read_text())["rows"] for f in spec.split(",")]


def mean(runs, i, key):
    v = [r[i][key] for r in runs if r[i].get(key) is not None]
    return statistics.fmean(v) if v else None


def fmt(x, nd=2):
    return "—" if x is None else f"{x:.{nd}f}"


def main():
    out, base, new = sys.argv[1], load(sys.argv[2]), load(sys.argv[3])
    lines = ["| ref line | block | EC | lost | encode call µs | encode kernel µs | encode kernel TB/s "
             "| decode call µs (round 5 → now) | decode kernel µs |",
             "|---|---|---|---|---|---|---|---|---|"]
    for i, r in enumerate(new[0]):
        S = r["stripes"]
        enc_bytes = S * (r["k"] + r["m"]) * r["block_B"]
        ek = mean(new, i, "enc_kernel_ns")
        dk = mean(new, i, "dec_kernel_ns")
        dec = (f"{fmt(mean(base, i, 'dec_call_us'))} → {fmt(mean(new, i, 'dec_call_us'))}"
               if r["lost"] else f"{fmt(mean(new, i, 'dec_call_us'))} (no loss: host scan only)")
        lines.append(f"| {r['ref_line']} | {r['block_B'] >> 10} KiB | {r['EC']} | {r['lost']} | "
                     f"{fmt(mean(new, i, 'enc_call_us'))} | {fmt(ek / 1e3 if ek else None)} | "
                     f"{fmt(enc_bytes / ek / 1e3 if ek else None)} | {dec} | "
                     f"{fmt(dk / 1e3 if dk else None)} |")
    Path(out).write_text("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
