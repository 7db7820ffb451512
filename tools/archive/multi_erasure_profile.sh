#!/bin/bash
# Kernel trace + per-counter PMC passes of the multi-erasure decode shapes
# (VERDICT r1 item 2): bench.py on each shape with its --lost, then
# tools/pmc_traffic.py turns gpurun_out/prof_<tag>/ into profiles/.
# Usage (inside gpurun): bash tools/archive/multi_erasure_profile.sh <round-tag>
set -euo pipefail
R=${1:?round tag}
for spec in "16,2,1048576,256 2" "16,8,65536,16384 8" "32,8,65536,8192 8" "16,4,65536,16384 4"; do
  set -- $spec
  W=$1; L=$2
  T="${R}_k$(echo $W | cut -d, -f1)m$(echo $W | cut -d, -f2)_lost$L"
  bash tools/gpu_profile.sh "$T" --workload "$W" --lost "$L" --steps 20 --warmup 5
done
