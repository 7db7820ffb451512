# Round-closing evidence at the last library: the round check (GPU tests,
# smoke, default bench, RCCL world-1 bench, timed-launch kernel stats) and the
# PMC traffic of the default bench's kernels (tools/gpu_profile.sh; turned
# into profiles/ by tools/pmc_traffic.py on the CPU side).
set -o pipefail
bash tools/round_check.sh ${1:-final} || exit 1
timeout -k 10 900 bash tools/gpu_profile.sh ${1:-final}_cfg3 > gpurun_out/${1:-final}/gpu_profile.log 2>&1 || { tail gpurun_out/${1:-final}/gpu_profile.log; exit 1; }
tail -1 gpurun_out/${1:-final}/gpu_profile.log
