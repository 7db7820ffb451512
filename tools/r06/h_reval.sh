#!/bin/bash
# Round 6, the final library's one full re-validation (VERDICT r05 item 6:
# at most one, since kernel code changed): tools/revalidate.sh (random GPU fuzz
# cases, big round trips, pipeline round trips, harness configs, a soak, the
# default bench); the RCCL 112-op group and world-1 topology tests; and the
# 8 MiB rows with losses once more, round 5 against the shipped library,
# alternating.  Output: gpurun_out/$1/.
set -euo pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl_p2p.py tests/test_bench_contract.py -x -v \
  --timeout 300 --timeout-method thread -k "rccl" > $O/pytest_rccl.log 2>&1 || { tail -30 $O/pytest_rccl.log; exit 1; }
tail -3 $O/pytest_rccl.log
bash tools/revalidate.sh $T 80000
for R in a b c; do
  timeout -k 10 400 python3 tools/small_msg_profile.py --out $O/small_r5$R.json --tag r5$R --lib tools/ab/r5 > $O/small_r5$R.log 2>&1
  timeout -k 10 400 python3 tools/small_msg_profile.py --out $O/small_wt$R.json --tag wt$R > $O/small_wt$R.log 2>&1
done
grep "lost=[1-9]" $O/small_r5?.log $O/small_wt?.log
echo "r06h done"
