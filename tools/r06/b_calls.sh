#!/bin/bash
# Round 6, second GPU call: the GPU suite on the working tree's library
# (kernel-argument capacities, single-pass host scan, topology record), then
# per-call latency at 8 MiB messages, round-5 library (tools/ab/r5) against the
# working tree's, and the 24 reference rows again.  Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs \
  > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -8 $O/pytest_gpu.log
for SH in "8 4 1024 1024" "32 8 1024 256" "16 8 1024 512" "16 1 1024 512"; do
  for R in 1 2; do
    LD_LIBRARY_PATH=$PWD/tools/ab/r5 timeout -k 10 120 tools/latency/latency 0 $SH 2000 >> $O/latency_r5.log 2>&1
    timeout -k 10 120 tools/latency/latency 0 $SH 2000 >> $O/latency_wt.log 2>&1
  done
done
grep -E "mode|decode auto|call only|arg" $O/latency_r5.log | head -60
grep -E "mode|decode auto|call only|arg" $O/latency_wt.log | head -60
timeout -k 10 400 python3 tools/small_msg_profile.py --out $O/small_wt.json --tag wt > $O/small_wt.log 2>&1
grep "lost=[1-9]" $O/small_wt.log
echo "r06b done"
