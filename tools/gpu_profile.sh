#!/bin/bash
# Profile bench.py on the GPU box: kernel trace + stats of the timed launches
# only (bench.py pauses the profiler outside xec.markers.timed_region, which
# rocprofv3 honours under --marker-trace), then one PMC pass per counter group
# (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).  PMC passes may
# not carry --marker-trace (gpurun refuses the combination), so they run
# without the legs (--no-host-pipeline): every remaining launch -- set-up,
# timed, verification -- has the headline shape and the same bytes.
# Usage (inside gpurun): bash tools/gpu_profile.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
# the library this profile measures (its source hash: erasure-code-benchmark_amd/Makefile)
python3 -c "import sys; sys.path.insert(0, 'erasure-code-benchmark_amd'); import xec; print(xec.build_info())" \
  > "$OUT/build_info.txt"
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d "$OUT/trace" -o kt --output-format csv \
  -- python3 bench.py --no-cpu-baseline "$@" > "$OUT/bench_trace.log" 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d "$OUT/pmc_$C" -o pmc --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-host-pipeline --no-verify --steps 5 --warmup 2 "$@" > "$OUT/bench_$C.log" 2>&1
done
echo "profile $TAG done"
