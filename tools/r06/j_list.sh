#!/bin/bash
# Round 6: where the 8 MiB decodes with losses spend their host time.  Rows
# 1123-1126 through bin/xec_bench (call times only), four libraries in
# rotation, four rounds: round 5 (tools/ab/r5), the shipped tree (first scan
# lists up to one lost block per stripe), a
# first-pass list of up to 1,024 (fulllist).  Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
for R in 1 2 3 4; do
  for L in r5 fulllist wt; do
    LIB=""; [ $L != wt ] && LIB="--lib tools/ab/$L"
    timeout -k 10 200 python3 tools/small_msg_profile.py --out $O/small_${L}_$R.json --tag ${L}_$R $LIB \
      --lines 1123,1124,1125,1126 --no-prof --iters 500 --warmup 50 > $O/small_${L}_$R.log 2>&1
  done
done
python3 - <<'PY'
import json, statistics as st, glob
O = "gpurun_out/" + __import__("sys").argv[1] if len(__import__("sys").argv) > 1 else None
PY
for L in r5 fulllist wt; do echo "== $L"; cat $O/small_${L}_*.log | sort; done
echo "r06j done"
