# One GPU call's worth of round-end checks: GPU tests, smoke, default bench,
# RCCL world-1 bench, and the default bench's kernel stats over the timed
# region only (rocprofv3 --marker-trace honours bench.py's markers.timed_region).
set -o pipefail
o=gpurun_out/${1:-r03}; mkdir -p $o
export TMPDIR=/tmp
{ nproc; python -c 'import os; print("affinity", len(os.sched_getaffinity(0)))'; cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; } > $o/host_cpus.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.txt 2>&1 || { tail -30 $o/pytest_gpu.txt; exit 1; }
tail -2 $o/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.txt 2>&1 || { tail $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
timeout -k 10 300 python -u bench.py > $o/bench_default.log 2>&1 || { tail $o/bench_default.log; exit 1; }
timeout -k 10 300 python -u bench.py --dist-world1 --no-cpu-baseline > $o/bench_world1_rccl.log 2>&1 || { tail $o/bench_world1_rccl.log; exit 1; }
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d $o/prof_timed -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > $o/bench_prof_timed.log 2>&1 || { tail $o/bench_prof_timed.log; exit 1; }
grep -o '"value": [0-9.]*' $o/bench_default.log $o/bench_world1_rccl.log
