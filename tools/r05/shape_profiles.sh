#!/bin/bash
# The DESIGN §3 table's multi-parity rows re-profiled on the shipped library
# (round 3's profiles were of earlier builds): timed-launch kernel stats and
# both PMC passes per shape and loss count, tags <prefix>_<k>_<m>_<bs>_l<lost>.
# Usage (inside gpurun): bash tools/r05/shape_profiles.sh <tag prefix>
set -euo pipefail
T=${1:?tag prefix}
while read -r W L; do
  tag=${T}_$(echo "$W" | cut -d, -f1-3 | tr , _)_l$L
  bash tools/gpu_profile.sh "$tag" --workload "$W" --lost "$L" --no-host-pipeline --steps 20 --warmup 5
done <<'SHAPES'
16,8,65536,16384 1
16,8,65536,16384 8
16,4,65536,16384 1
16,4,65536,16384 4
32,8,65536,8192 1
32,8,65536,8192 8
16,2,1048576,256 1
16,2,1048576,256 2
32,4,1048576,256 1
SHAPES
echo "shape profiles done"
