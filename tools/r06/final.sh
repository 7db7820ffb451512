#!/bin/bash
# Round 6's final library, one GPU call: configs 3, 2, 4 re-profiled (timed-
# launch kernel stats + one PMC pass per counter, tools/gpu_profile.sh, which
# records the library's build id), then the round-end checks the driver runs:
# the whole GPU suite, smoke(), the default bench line; and the one-GPU
# rehearsals of the N > 1 paths (RCCL at world 1, the multi-device leg over a
# repeated device list).  Output: gpurun_out/$1/ and gpurun_out/prof_$1_<cfg>/.
set -euo pipefail
T=${1:?tag}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for W in cfg3 cfg2 cfg4; do
  timeout -k 10 600 bash tools/gpu_profile.sh ${T}_$W --workload $W --steps 20 --warmup 5
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs \
  > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
tail -c 300 $O/bench.json
timeout -k 10 300 python3 bench.py --dist-world1 --no-cpu-baseline --multi-devices 0,0 \
  > $O/bench_world1_multi.json 2> $O/bench_world1_multi.err
XEC_FUZZ_CASES=2500 XEC_FUZZ_SEED=92000 timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread > $O/pytest_fuzz.txt 2>&1 || { tail -30 $O/pytest_fuzz.txt; exit 1; }
tail -1 $O/pytest_fuzz.txt
echo "final done"
