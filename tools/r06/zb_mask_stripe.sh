#!/bin/bash
# Argument masks over stripe tiles (batches of <= 1,024 stripes with a few
# losses per stripe, past the 1,024-entry list): the GPU tests they touch; the
# call against the library before the masks (tools/ab/shipped) at an 8 MiB
# class-tile shape and a 16 MiB stripe-tile shape (tools/latency); and stripe
# tiles over the bitmap (1) against the masks (4) in one process at two 64 KiB
# shapes (tools/ab/ab.py).  Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -rs \
  tests/test_gpu_parity.py tests/test_gpu_stream_lifetime.py tests/test_gpu_upload_stress.py \
  tests/test_plugin_harness.py tests/test_gpu_fuzz.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for R in 1 2; do
  for L in shipped wt; do
    LP=""; [ $L != wt ] && LP=$PWD/tools/ab/$L
    for shape in "32 8 1024 256 8" "16 8 1024 1024 2"; do
      set -- $shape
      LD_LIBRARY_PATH=$LP${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} timeout -k 10 120 \
        tools/latency/latency 0 $1 $2 $3 $4 500 $5 > $O/lat_${L}_${1}_${2}_l$5_$R.log 2>&1
    done
  done
done
grep -H "decode auto + sync" $O/lat_*.log
while read -r W Lo; do
  timeout -k 10 300 python3 tools/ab/ab.py --libs wt --workload $W --lost $Lo --tilings 1,4 \
    --rounds 7 --iters 10 > $O/ab_$(echo $W | tr , _)_l$Lo.log 2>&1 || { tail -20 $O/ab_*_l$Lo.log; exit 1; }
  tail -2 $O/ab_$(echo $W | tr , _)_l$Lo.log
done <<'SHAPES'
16,8,65536,1000 2
32,8,65536,1000 2
SHAPES
echo "zb done"
