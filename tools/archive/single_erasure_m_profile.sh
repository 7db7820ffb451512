#!/bin/bash
# Kernel trace + per-counter PMC passes of the single-erasure decodes at m > 1
# (DESIGN.md §3 "Single-erasure decode at m > 1"): bench.py on each shape with
# one lost data block per stripe; tools/pmc_traffic.py turns
# gpurun_out/prof_<tag>/ into profiles/.
# Usage (inside gpurun): bash tools/archive/single_erasure_m_profile.sh <round-tag>
set -euo pipefail
R=${1:?round tag}
for W in 16,4,65536,16384 16,8,65536,16384 32,8,65536,8192 16,2,1048576,256; do
  T="${R}_k$(echo $W | cut -d, -f1)m$(echo $W | cut -d, -f2)_lost1"
  bash tools/gpu_profile.sh "$T" --workload "$W" --lost 1 --steps 20 --warmup 5 --no-host-pipeline
done
