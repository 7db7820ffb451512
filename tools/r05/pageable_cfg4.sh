#!/bin/bash
# staged pageable decode at small blocks issued one copy per
# run of survivors; round 5 stages such chunks whole.  Config 4's shape and
# config 3's, round-4 final library (tools/ab/libxec_r4final.so) against the
# working tree's, alternating processes, 2 rounds.  Output: gpurun_out/r05j/.
# tools/ab/libxec_r4final.so (git-ignored) is rebuilt from commit 02ed769:
#   git worktree add /tmp/r4 02ed769 && make -C /tmp/r4/erasure-code-benchmark_amd \
#     && cp /tmp/r4/erasure-code-benchmark_amd/xec/libxec_hip.so tools/ab/libxec_r4final.so
set -euo pipefail
O=gpurun_out/r05j
mkdir -p $O
for R in 1 2; do
  for L in tools/ab/libxec_r4final.so erasure-code-benchmark_amd/xec/libxec_hip.so; do
    XEC_LIB=$L timeout -k 10 200 python3 tools/pageable_probe.py --shape 32,1,4096 --stripes 8192 \
      --chunk 1024 --kinds pinned,pageable >> $O/cfg4.log 2>&1
    XEC_LIB=$L timeout -k 10 200 python3 tools/pageable_probe.py --kinds pageable >> $O/cfg3.log 2>&1
  done
done
echo "r05j done"
