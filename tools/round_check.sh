set -o pipefail
o=gpurun_out/${1:-r02aw}; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.txt 2>&1 || { tail -20 $o/pytest_gpu.txt; exit 1; }
tail -2 $o/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.txt 2>&1 || { tail $o/smoke.txt; exit 1; }
tail -1 $o/smoke.txt
timeout -k 10 300 python -u bench.py > $o/bench_default.log 2>&1 || { tail $o/bench_default.log; exit 1; }
timeout -k 10 300 python -u bench.py --dist-world1 --no-cpu-baseline > $o/bench_world1_rccl.log 2>&1 || { tail $o/bench_world1_rccl.log; exit 1; }
grep -o '"value": [0-9.]*' $o/bench_default.log $o/bench_world1_rccl.log
