#!/bin/bash
# The distinct-GPU test programs, rehearsed at world 1 on the one-GPU box so a
# mistake in them shows before the 8-GPU node runs them: the RCCL multi-rank
# script of tests/test_gpu_multi_rank.py under torch.distributed.run with one
# rank (scatter to itself, encode, gather), and the multi-device leg at the
# distinct-device test's shape over one device.  Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
(cd tests && python3 -c "import sys; sys.path.insert(0, '.'); import test_gpu_multi_rank as t; open('/tmp/multi_rank_script.py', 'w').write(t.SCRIPT)")
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 /tmp/multi_rank_script.py erasure-code-benchmark_amd 256 > $O/multi_rank_world1.log 2>&1
grep '^{' $O/multi_rank_world1.log
timeout -k 10 300 erasure-code-benchmark_amd/bin/xec_multi_leg --devices 0 --stripes-per-device 256 --data 16 \
  --parity 1 --block 1M --iterations 3 --warmup 1 --scatter-reps 1 > $O/leg_one.json
head -c 600 $O/leg_one.json
echo "r06r done"
