set -o pipefail
o=gpurun_out/r03g; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.txt 2>&1 || { tail -30 $o/pytest_gpu.txt; exit 1; }
tail -2 $o/pytest_gpu.txt
timeout -k 10 600 python -u tools/lab/mix_ceiling.py --out $o/mix_ceiling.json > $o/mix_ceiling.log 2>&1 || { tail $o/mix_ceiling.log; exit 1; }
for w in cfg3 cfg4 cfg2; do timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-host-pipeline > $o/bench_$w.log 2>&1 || { tail $o/bench_$w.log; exit 1; }; done
grep -ho '"value": [0-9.]*\|"decode_ms": [0-9.]*\|"encode_ms": [0-9.]*' $o/bench_*.log
