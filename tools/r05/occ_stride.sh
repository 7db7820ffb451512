#!/bin/bash
# Residency by member stride (follow-up of r05d: the read-only ceiling of 8
# members 4 MiB apart is 2 % higher uncapped than at the 4 waves per SIMD the
# library picks for 8 members).  Encode + decode per xec_set_occupancy value,
# interleaved, at 8-member shapes whose member stride m*bs is 1, 2, 4 MiB and
# 64 KiB.  Output: gpurun_out/r05e/.
set -euo pipefail
O=gpurun_out/r05e
mkdir -p $O
for SH in 32,4,1048576,256 16,2,1048576,256 8,1,1048576,512 16,2,2097152,128 8,1,65536,8192 32,4,65536,4096; do
  for P in select rotating; do
    timeout -k 10 180 python3 tools/lab/shape_profile.py --shape $SH --pattern $P --occ 0,8,6,3,2 \
      --iters 10 --rounds 5 >> $O/occ.log 2>&1
  done
done
echo "r05e done"
