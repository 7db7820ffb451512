#!/bin/bash
# configs 2-4 re-profiled on HEAD's library in one
# session -- timed-launch kernel stats and both PMC passes per workload
# (tools/gpu_profile.sh records the library's build id beside them).
# Usage: bash tools/r05/profiles.sh <tag prefix> [workloads...]
set -euo pipefail
T=${1:?tag prefix}; shift
WS=${*:-cfg3 cfg2 cfg4}
for W in $WS; do
  bash tools/gpu_profile.sh ${T}_$W --workload $W --steps 20 --warmup 5
done
echo "profiles done"
