#!/bin/bash
# Refresh of DESIGN.md §3's per-shape table at the round's last
# library: timed-launch kernel stats + PMC traffic (tools/gpu_profile.sh) of
# the given shapes; tools/pmc_traffic.py turns gpurun_out/prof_<tag>/ into
# profiles/.  Shapes are "workload:lost" (bench.py workload name or k,m,bs,S).
# Usage (inside gpurun): bash tools/archive/shape_table.sh <round-tag> <shape>...
set -euo pipefail
R=${1:?round tag}; shift
for spec in "$@"; do
  W=${spec%%:*}; L=${spec##*:}
  T="${R}_$(echo "$W" | tr , _)_lost$L"
  bash tools/gpu_profile.sh "$T" --workload "$W" --lost "$L" --steps 20 --warmup 5 --no-host-pipeline
done
