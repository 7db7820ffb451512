#!/bin/bash
# Loss masks uploaded in place of the bitmap (decode_mask_kernel, S > 1,024,
# k <= 32): the GPU tests they touch; then, in one process, stripe / class
# tiles over the bitmap (1 / 2) against the automatic choice (0: the masks) at
# config 4, the DESIGN §3 table's multi-erasure shapes past 1,024 stripes and
# two 64 KiB shapes with two losses per stripe (tools/ab/ab.py).
# Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -rs \
  tests/test_gpu_parity.py tests/test_gpu_stream_lifetime.py tests/test_gpu_upload_stress.py \
  tests/test_plugin_harness.py tests/test_gpu_fuzz.py tests/test_gpu_drop_in.py > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
while read -r W Lo T; do
  timeout -k 10 300 python3 tools/ab/ab.py --libs wt --workload $W --lost $Lo --tilings $T \
    --rounds 7 --iters 10 > $O/ab_$(echo $W | tr , _)_l$Lo.log 2>&1 || { tail -20 $O/ab_*_l$Lo.log; exit 1; }
  echo "== $W lost $Lo"; tail -3 $O/ab_$(echo $W | tr , _)_l$Lo.log
done <<'SHAPES'
cfg4 1 1,0
16,8,65536,16384 1 1,0
16,4,65536,16384 1 1,0
32,8,65536,8192 1 1,0
16,4,65536,16384 4 2,0
16,8,65536,16384 8 2,0
16,8,65536,4096 2 1,0
SHAPES
echo "zc done"
