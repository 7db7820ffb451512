set -o pipefail
o=gpurun_out/r03d; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.txt 2>&1 || { tail -30 $o/pytest_gpu.txt; exit 1; }
tail -2 $o/pytest_gpu.txt
timeout -k 10 900 bash tools/gpu_profile.sh r03d || exit 1
cat gpurun_out/prof_r03d/trace/kt_kernel_stats.csv | cut -c1-200
