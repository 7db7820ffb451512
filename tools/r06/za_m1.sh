#!/bin/bash
# Would device-memory loss masks help config 4 (32+1, stripe tiles over the
# bitmap)?  Stripe tiles (1), the work list (3, in the arguments here) and the
# argument masks (4) in one process at config 4's stripe shape with S = 1,024
# (the masks' limit), and at 16+4 x 64 KiB with one loss per stripe.
# Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
while read -r W L; do
  timeout -k 10 300 python3 tools/ab/ab.py --libs wt --workload $W --lost $L --tilings 1,3,4 \
    --rounds 7 --iters 20 > $O/ab_$(echo $W | tr , _)_l$L.log 2>&1 || { tail -20 $O/ab_*_l$L.log; exit 1; }
  tail -3 $O/ab_$(echo $W | tr , _)_l$L.log
done <<'SHAPES'
32,1,4096,1024 1
32,1,65536,1024 1
16,4,65536,1024 1
SHAPES
echo "za done"
