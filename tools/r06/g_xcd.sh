#!/bin/bash
# Round 6 experiment: XCD-grouped tile order (tools/ab/patches/xcd_group.py,
# G = 2 / 4 / 8 consecutive 1 KiB tiles per XCD) against the working tree,
# one process per shape, interleaved rounds.  Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
for W in cfg3 cfg2 cfg4 16,4,65536,16384 16,2,1048576,256; do
  timeout -k 10 300 python3 tools/ab/ab.py --libs wt6f,xg2,xg4,xg8 --workload $W --rounds 5 \
    >> $O/xcd_group.log 2>&1
done
grep -v amdgpu $O/xcd_group.log
echo "r06g done"
