#!/bin/bash
# The pipeline's small-block decode (round 5): whole-chunk inputs and gathered
# outputs.  Pipeline + error-state GPU tests, then config 4's and config 3's
# shapes through tools/pageable_probe.py, round-4 final library against the
# working tree's, alternating processes.  Output: gpurun_out/$1/.
# tools/ab/libxec_r4final.so (git-ignored) is rebuilt from commit 02ed769:
#   git worktree add /tmp/r4 02ed769 && make -C /tmp/r4/erasure-code-benchmark_amd \
#     && cp /tmp/r4/erasure-code-benchmark_amd/xec/libxec_hip.so tools/ab/libxec_r4final.so
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_pipeline.py tests/test_gpu_error_state.py tests/test_gpu_stream_lifetime.py > $O/pytest.log 2>&1
tail -1 $O/pytest.log
for R in 1 2; do
  for L in ${LIBS:-tools/ab/libxec_r4final.so erasure-code-benchmark_amd/xec/libxec_hip.so}; do
    XEC_LIB=$L timeout -k 10 200 python3 tools/pageable_probe.py --shape 32,1,4096 --stripes 8192 \
      --chunk 1024 --kinds pinned,pageable >> $O/cfg4.log 2>&1
    XEC_LIB=$L timeout -k 10 200 python3 tools/pageable_probe.py --shape 8,1,65536 --stripes 1024 \
      --chunk 128 --kinds pinned,pageable >> $O/cfg2.log 2>&1
    XEC_LIB=$L timeout -k 10 200 python3 tools/pageable_probe.py --kinds pinned,pageable >> $O/cfg3.log 2>&1
    XEC_LIB=$L timeout -k 10 200 python3 tools/pageable_probe.py --shape 16,4,65536 --stripes 1024 \
      --chunk 64 --kinds pinned,pageable >> $O/s16p4_64k.log 2>&1
    XEC_LIB=$L timeout -k 10 200 python3 tools/pageable_probe.py --shape 16,2,262144 --stripes 256 \
      --chunk 32 --kinds pinned,pageable >> $O/s16p2_256k.log 2>&1
  done
done
echo "pipeline_small done"
