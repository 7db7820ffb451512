#!/bin/bash
# Round 6: the shipped library's decode paths under random shapes (the host
# scan's listing changed after the full re-validation): 2,500 GPU fuzz cases,
# 300 big round trips; and the reference's 53 published GPU rows again
# (tools/reference_compare.py).  Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
export TMPDIR=/tmp
XEC_FUZZ_CASES=2500 XEC_FUZZ_SEED=91000 timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py -x -q \
  --timeout 300 --timeout-method thread > $O/pytest_fuzz.txt 2>&1 || { tail -30 $O/pytest_fuzz.txt; exit 1; }
tail -1 $O/pytest_fuzz.txt
timeout -k 10 300 python -u tools/fuzz_big.py --cases 300 --seed 91001 --out $O/fuzz_big.json > $O/fuzz_big.log 2>&1
tail -1 $O/fuzz_big.log
timeout -k 10 600 python -u tools/reference_compare.py --out $O/reference_compare.json > $O/reference_compare.log 2>&1
tail -5 $O/reference_compare.log
echo "r06l done"
