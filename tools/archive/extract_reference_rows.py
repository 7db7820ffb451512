#!/usr/bin/env python3
"""Regenerate tools/reference_gpu_rows.csv: every "XOR-EC (GPU Computation)"
row of the reference's published results/raw/final_results.csv (all 20
columns, prefixed with the file line number).  Data extraction only; runs
where /root/reference is mounted (this container), never on the GPU box."""
from pathlib import Path

SRC = Path("/root/reference/results/raw/final_results.csv")
DST = Path(__file__).resolve().parent / "reference_gpu_rows.csv"


def main():
    lines = SRC.read_text().splitlines()
    out = ["# Published GPU rows of the reference: results/raw/final_results.csv, every",
           "# \"XOR-EC (GPU Computation)\" row (kenji-k6/erasure-code-benchmark, Tesla V100,",
           "# 500 iterations after 100 warm-up), with their file line numbers. Data only;",
           "# regenerate with tools/archive/extract_reference_rows.py.",
           "line," + lines[0]]
    out += [f"{i},{ln}" for i, ln in enumerate(lines[1:], start=2)
            if ln.startswith('"XOR-EC (GPU Computation)"')]
    DST.write_text("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
