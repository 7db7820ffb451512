#!/bin/bash
# The latency probes at 32+4 x 1 KiB (8 MiB) plainly and under rocprofv3
# --kernel-trace --stats, so the profiler's durations of an empty kernel, a
# 4-byte store, the copy probe and the codec's kernels sit in one table.
# Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/latency/latency 0 32 4 1024 256 500 > $O/probe_32_4.log 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o kt --output-format csv -- \
  tools/latency/latency 0 32 4 1024 256 500 > $O/probe_32_4_prof.log 2>&1
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
cut -d, -f1-8 $O/kernel_stats.csv | cut -c1-160
