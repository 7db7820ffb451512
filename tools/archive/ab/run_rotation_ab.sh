#!/bin/bash
# Rotation by run position (tools/archive/ab/patches/run_rotation.py) against the
# product's rotation by stripe index, in one process per shape and pattern:
# each lib with no rotation (-1) and with R = 3 KiB (the automatic choice's R).
# Usage (inside gpurun): bash tools/archive/ab/run_rotation_ab.sh <out-dir>
set -euo pipefail
o=${1:?out dir}; mkdir -p "$o"
for w in 16,2,1048576,256 8,2,1048576,256 16,4,1048576,256 32,4,1048576,256 16,2,524288,512; do
  for pat in random same rotating; do
    timeout -k 10 240 python -u tools/ab/ab.py --libs base,runrot --rotations=-1,3 \
      --workload $w --pattern $pat --rounds 5 --iters 8 --out "$o/rr_${w//,/_}_$pat.json"
  done
done
