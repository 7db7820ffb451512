#!/bin/bash
# Round 6, fourth GPU call: the 8 MiB rows and per-call latency, round-5
# library (tools/ab/r5) against the working tree's, alternating processes so a
# process's placement cannot pass for a library difference.  Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
export TMPDIR=/tmp
for R in a b; do
  timeout -k 10 400 python3 tools/small_msg_profile.py --out $O/small_r5$R.json --tag r5$R --lib tools/ab/r5 > $O/small_r5$R.log 2>&1
  timeout -k 10 400 python3 tools/small_msg_profile.py --out $O/small_wt$R.json --tag wt$R > $O/small_wt$R.log 2>&1
done
for SH in "8 4 1024 1024 2000 1" "32 8 1024 256 2000 1" "32 8 1024 256 2000 2" "32 8 1024 256 2000 4" "32 8 1024 256 2000 8" "16 1 1024 512 2000 1"; do
  for R in 1 2; do
    LD_LIBRARY_PATH=$PWD/tools/ab/r5 timeout -k 10 120 tools/latency/latency 0 $SH >> $O/latency_r5.log 2>&1
    timeout -k 10 120 tools/latency/latency 0 $SH >> $O/latency_wt.log 2>&1
  done
done
echo "r06d done"
