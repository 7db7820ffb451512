# Re-validation of the current library: randomised GPU campaigns, a soak and a
# default bench (randomised campaigns with a tag and a seed base of their own).
# Usage (inside gpurun): bash tools/revalidate.sh <tag> <seed-base>
set -o pipefail
t=${1:?tag}; s=${2:?seed base}
o=gpurun_out/$t; mkdir -p $o
export TMPDIR=/tmp
XEC_FUZZ_CASES=2500 XEC_FUZZ_SEED=$s timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > $o/pytest_fuzz_2500.txt 2>&1 || { tail -30 $o/pytest_fuzz_2500.txt; exit 1; }
tail -1 $o/pytest_fuzz_2500.txt
timeout -k 10 300 python -u tools/fuzz_big.py --cases 300 --seed $((s + 1)) --out $o/fuzz_big.json > $o/fuzz_big.log 2>&1 || { tail $o/fuzz_big.log; exit 1; }
tail -1 $o/fuzz_big.log
timeout -k 10 300 python -u tools/fuzz_big.py --pipeline --cases 100 --seed $((s + 2)) --out $o/fuzz_big_pipeline.json > $o/fuzz_big_pipeline.log 2>&1 || { tail $o/fuzz_big_pipeline.log; exit 1; }
tail -1 $o/fuzz_big_pipeline.log
timeout -k 10 300 python -u tools/fuzz_harness.py --cases 40 --seed $((s + 3)) --out $o/fuzz_harness.json > $o/fuzz_harness.log 2>&1 || { tail $o/fuzz_harness.log; exit 1; }
tail -1 $o/fuzz_harness.log
timeout -k 10 200 python -u tools/soak.py --seconds 120 --out $o/soak.json > $o/soak.log 2>&1 || { tail $o/soak.log; exit 1; }
tail -1 $o/soak.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench.log 2>&1 || { tail $o/bench.log; exit 1; }
grep -o '"value": [0-9.]*' $o/bench.log
