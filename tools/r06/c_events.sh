#!/bin/bash
# Round 6, third GPU call: kernel timing from each launch's own dispatch
# (xec_set_kernel_events) against packet events between kernels, in the
# default bench line; the reference's 8 MiB rows, round-5 library against the
# working tree's on one box.  Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernel_events.py tests/test_bench_contract.py \
  tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "kernel_events or bench or capacities or policy or tilings_bit" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for R in 1 2 3; do
  for E in dispatch packets; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-host-pipeline --kernel-events $E \
      > $O/bench_${E}_$R.json 2> $O/bench_${E}_$R.err
    python3 -c "import json,sys; d=json.load(open('$O/bench_${E}_$R.json')); r=d['roofline']; print('$E', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_ms'], r.get('rocprof_profile',{}).get('over_hip_events_ms'), d['roofline_by_kernel']['encode']['avg_launch_ms'])"
  done
done
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d $O/prof_dispatch -o kt --output-format csv \
  -- python3 bench.py --no-cpu-baseline --no-host-pipeline > $O/bench_prof_dispatch.json 2> $O/bench_prof_dispatch.err
python3 -c "import json; d=json.load(open('$O/bench_prof_dispatch.json')); print('under rocprof', d['roofline']['avg_launch_ms'], d['roofline_by_kernel']['encode']['avg_launch_ms'])"
cat $(find $O/prof_dispatch -name '*kernel_stats.csv')
timeout -k 10 400 python3 tools/small_msg_profile.py --out $O/small_r5.json --tag r5 --lib tools/ab/r5 > $O/small_r5.log 2>&1
timeout -k 10 400 python3 tools/small_msg_profile.py --out $O/small_wt.json --tag wt > $O/small_wt.log 2>&1
grep -v amdgpu $O/small_r5.log $O/small_wt.log
echo "r06c done"
