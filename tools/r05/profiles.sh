#!/bin/bash
# configs 2-4 re-profiled on HEAD's library in one
# session -- timed-launch kernel stats and both PMC passes per workload
# (tools/gpu_profile.sh records the library's build id beside them).
set -euo pipefail
for W in cfg3 cfg2 cfg4; do
  bash tools/gpu_profile.sh r05g_$W --workload $W --steps 20 --warmup 5
done
echo "profiles done"
