#!/usr/bin/env python3
"""In-container check that the CPU restatement is as fast as the reference.

SURVEY.md §8(d): before the restatement (oracle/xorec_oracle.c, "kind": "port")
is timed as the CPU baseline on the GPU box, check here that its speed is
within ~10 % of the reference's own CPU code (src/xorec/xorec.cpp compiled
unmodified into oracle/_ref/ref_driver by `make -C oracle ref`) at the same
thread count, on the same loop (xorec_bm.cpp:27-58: OpenMP parallel-for over
stripes, encode then single-erasure decode) and the same batch shape.  Runs
only where /root/reference was built (this container); bench.py never runs
ref_driver.

    python tools/cpu_port_vs_ref.py [--seconds 8] [--out profiles/r02_cpu_port_vs_ref.json]
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import bench  # noqa: E402
import xorec_oracle as xo  # noqa: E402


ROUNDS = 4


def ref_rate(k, m, bs, S, threads, seconds, version):
    drv = ROOT / "oracle" / "_ref" / "ref_driver"
    p = subprocess.run([str(drv), "bench", str(k), str(m), str(bs), str(S), str(version),
                        str(threads), str(seconds)], capture_output=True, text=True, check=True)
    r = dict(line.split(" ", 1) for line in p.stdout.strip().splitlines())
    assert int(r["fail"]) == 0
    b_enc, b_dec = bench.algorithmic_bytes(S, k, m, bs)
    return int(r["reps"]) * (b_enc + b_dec) / float(r["seconds"]) / 1e9, int(r["reps"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r02_cpu_port_vs_ref.json"))
    a = ap.parse_args()
    o = xo.COracle()
    threads_all = bench._host_threads()[0]  # nproc
    _, avx512 = bench._cpu_model()
    version = 3 if avx512 else 2
    rows = []
    for name, (k, m, bs, _, _) in bench.WORKLOADS.items():
        S = max(1, (1 << 30) // (k * bs))  # 1 GiB of data (this container has 64 GiB)
        for threads in (threads_all, 1):
            secs = a.seconds if threads > 1 else a.seconds / 2
            # interleave ref, port, ref, port, ... -> best of ROUNDS each (this
            # container shares its cores; single runs spread by +-20 %)
            rr, pp = [], []
            for _ in range(ROUNDS):
                rr.append(ref_rate(k, m, bs, S, threads, secs / ROUNDS, version)[0])
                pp.append(bench.cpu_time_port(o, xo, k, m, bs, S, secs / ROUNDS, threads)[0])
            ref, port = max(rr), max(pp)
            row = {"workload": name, "k": k, "m": m, "bs": bs, "stripes": S, "threads": threads,
                   "reference_GBps": round(ref, 2), "port_GBps": round(port, 2),
                   "port_over_reference": round(port / ref, 3),
                   "runs": {"reference": [round(x, 2) for x in rr],
                            "port": [round(x, 2) for x in pp]}}
            print(json.dumps(row), flush=True)
            rows.append(row)
    out = {"what": "oracle/xorec_oracle.c (port) vs reference src/xorec compiled unmodified "
                   "(oracle/_ref/ref_driver), same loop (xorec_bm.cpp:27-58), same shapes, "
                   f"algorithmic GB/s of encode + single-erasure decode, best of {ROUNDS} interleaved",
           "reference_version": "AVX512" if version == 3 else "AVX2",
           "cpu_model": bench._cpu_model()[0], "rows": rows}
    Path(a.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
