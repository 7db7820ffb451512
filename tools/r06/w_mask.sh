#!/bin/bash
# Kernel-argument loss masks (decode_argmask_kernel): the GPU tests they touch on
# the new library, then the reference's rows 1123-1126 (bin/xec_bench, call
# times) and three small multi-erasure shapes (tools/latency) on the shipped
# library (tools/ab/shipped, 8fc0bbdaaab2f1cb) and the new one, alternating.
# Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -rs \
  tests/test_gpu_parity.py tests/test_gpu_stream_lifetime.py tests/test_gpu_upload_stress.py \
  tests/test_plugin_harness.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for R in 1 2 3; do
  for L in shipped wt; do
    LIB=""; [ $L != wt ] && LIB="--lib tools/ab/$L"
    timeout -k 10 200 python3 tools/small_msg_profile.py --out $O/small_${L}_$R.json --tag ${L}_$R $LIB \
      --lines 1123,1124,1125,1126 --no-prof --iters 500 --warmup 50 > $O/small_${L}_$R.log 2>&1
    LP=""; [ $L != wt ] && LP=$PWD/tools/ab/$L
    for shape in "32 8 1024 256 8" "16 4 1024 512 4" "8 4 1024 1024 4"; do
      set -- $shape
      LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 120 \
        tools/latency/latency 0 $1 $2 $3 $4 500 $5 > $O/lat_${L}_${1}_${2}_$R.log 2>&1
    done
  done
done
for L in shipped wt; do echo "== $L"; cat $O/small_${L}_*.log | sort; grep -h "decode auto + sync" $O/lat_${L}_*; done
echo "r06w done"
