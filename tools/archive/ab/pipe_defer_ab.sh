# Host-in/host-out pipeline: outputs queued behind the next chunk's inputs
# (tree) against outputs right behind their own kernel (libxec_pipe_before.so),
# pinned and pageable host buffers, two alternations per library.
set -e
out=gpurun_out/${1:-r03w}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $out/pytest_pipeline.txt 2>&1
tail -1 $out/pytest_pipeline.txt
for rep in 1 2; do
  for lib in before tree; do
    if [ $lib = before ]; then export XEC_LIB=$PWD/tools/ab/libxec_pipe_before.so; else unset XEC_LIB; fi
    timeout -k 10 300 python -u tools/pageable_probe.py --stripes 64 --reps 5 --kinds pinned,pageable,data_pageable_parity_pinned --out $out/pageable_${lib}_$rep.json > $out/pageable_${lib}_$rep.log 2>&1
    echo "$lib $rep"; grep -v amdgpu.ids $out/pageable_${lib}_$rep.log
  done
done
