#!/bin/bash
# Round 6, first GPU call:
#  * kernel ns vs call us at the reference's 8 MiB messages (tools/small_msg_profile.py),
#    round-5 library (tools/ab/r5) and the working tree's (kernel-argument lists sized
#    to their entries);
#  * per-call latency (tools/latency), both libraries;
#  * configs 2-4 encode/decode, both libraries in one process (tools/ab/ab.py);
#  * config 4's decode: stripe tiles against work-list tiles, one process, and
#    the work-list variant's PMC traffic (tools/gpu_profile.sh);
#  * the new capacity parity tests.
# Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_config5.py \
  tests/test_gpu_multi_rank.py tests/test_plugin_harness.py -x -v --timeout 300 --timeout-method thread \
  -k "capacities or tilings_bit_exact or policy or config5 or distinct or scatter" -rs > $O/pytest_parity.log 2>&1
tail -12 $O/pytest_parity.log
timeout -k 10 300 erasure-code-benchmark_amd/bin/xec_multi_leg --devices 0,0 --stripes-per-device 64 \
  --iterations 2 --warmup 1 > $O/leg_00.json
cat $O/leg_00.json | head -c 3000
for L in r5 wt; do
  LIBARG=""; [ $L = r5 ] && LIBARG="--lib tools/ab/r5"
  timeout -k 10 400 python3 tools/small_msg_profile.py --out $O/small_$L.json --tag $L $LIBARG > $O/small_$L.log 2>&1
  tail -2 $O/small_$L.log
done
timeout -k 10 120 tools/latency/latency 0 8 4 1024 1024 2000 > $O/latency_wt.log 2>&1
LD_LIBRARY_PATH=$PWD/tools/ab/r5 timeout -k 10 120 tools/latency/latency 0 8 4 1024 1024 2000 > $O/latency_r5.log 2>&1
for W in cfg3 cfg2 cfg4; do
  timeout -k 10 200 python3 tools/ab/ab.py --libs r5final,wt6a --workload $W --rounds 5 >> $O/ab_r5_wt.log 2>&1
done
cat $O/ab_r5_wt.log
for SH in cfg4 16,8,65536,16384 32,8,65536,8192 16,4,65536,16384; do
  timeout -k 10 200 python3 tools/ab/ab.py --libs wt6a --workload $SH --tilings 1,3 --rounds 5 \
    >> $O/tiling_ab.log 2>&1
done
cat $O/tiling_ab.log
timeout -k 10 700 bash tools/gpu_profile.sh r06a_cfg4list --workload cfg4 --decode-tiling 3
mv gpurun_out/prof_r06a_cfg4list $O/
echo "r06a done"
