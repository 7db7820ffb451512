#!/bin/bash
# Launch knobs at the reference's 8 MiB shapes (tools/lab/small_launch.py), one
# process, variants interleaved.  Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 400 python3 -u tools/lab/small_launch.py --out $O/small_launch.json > $O/small_launch.log 2>&1 \
  || { tail -30 $O/small_launch.log; exit 1; }
tail -3 $O/small_launch.log | cut -c1-400
