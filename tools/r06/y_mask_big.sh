#!/bin/bash
# The argument-mask tiles at bandwidth scale: class (2), stripe (1) and mask (4)
# tiles in one process (tools/ab/ab.py --tilings) at the multi-erasure shapes the
# masks now take (S <= 1,024, k <= 32, several losses per stripe), and the DESIGN
# §3 table's 16+2 x 1 MiB x 256, 2 lost row re-profiled on the shipped library.
# Output: gpurun_out/$1/, gpurun_out/prof_$1_16_2_1048576_l2/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
while read -r W L; do
  timeout -k 10 300 python3 tools/ab/ab.py --libs wt --workload $W --lost $L --tilings 1,2,4 \
    --rounds 5 --iters 10 > $O/ab_$(echo $W | tr , _)_l$L.log 2>&1 || { tail -20 $O/ab_*_l$L.log; exit 1; }
  tail -4 $O/ab_$(echo $W | tr , _)_l$L.log
done <<'SHAPES'
16,2,1048576,256 2
8,2,1048576,512 2
16,4,65536,1024 4
16,8,65536,1024 8
32,8,65536,1024 8
SHAPES
bash tools/gpu_profile.sh ${1}_16_2_1048576_l2 --workload 16,2,1048576,256 --lost 2 --no-host-pipeline --steps 20 --warmup 5
echo "r06y done"
