# Uploads on the caller's stream when it is idle: GPU tests of the decode
# paths, the reference rows against the round-2 library, and the in-process
# r2-vs-tree A/B at config 4 and 16+8 (busy streams: side uploads kept).
set -o pipefail
o=gpurun_out/${1:-r03zl}; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_upload_stress.py tests/test_gpu_threads.py tests/test_gpu_pipeline.py tests/test_gpu_fuzz.py tests/test_gpu_decode_device.py -x -q --timeout 200 --timeout-method thread > $o/pytest.txt 2>&1 || { tail -30 $o/pytest.txt; exit 1; }
tail -1 $o/pytest.txt
bash tools/ab/refrows_ab.sh ${1:-r03zl} > $o/refrows.log 2>&1 || { tail $o/refrows.log; exit 1; }
for w in cfg4 16,8,65536,16384; do
  timeout -k 10 240 python -u tools/ab/ab.py --libs r2final,head --workload $w --rounds 7 --iters 10 --out $o/r2_vs_head_${w//,/_}.json 2>/dev/null | tail -2 || exit 1
done
