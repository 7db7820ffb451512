# Host-in/host-out decode at m > 1: the previous library (every survivor and
# parity travels) against the tree (only classes that lost a block travel).
set -e
out=gpurun_out/${1:-r02az}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $out/pytest_pipeline.txt 2>&1
tail -1 $out/pytest_pipeline.txt
for w in 16,4,1048576,256:1 16,4,1048576,256:2 16,8,65536,4096:1 16,1,1048576,256:1; do
  shape=${w%:*}; lost=${w#*:}
  for lib in old new; do
    if [ $lib = old ]; then export XEC_LIB=$PWD/tools/ab/libxec_pipe_old.so; else unset XEC_LIB; fi
    timeout -k 10 300 python -u tools/archive/host_pipeline.py --workload $shape --lost $lost --chunks 8 \
      --streams 3 --reps 5 --out $out/pipe_${lib}_${shape//,/_}_l$lost.json > $out/pipe_${lib}_${shape//,/_}_l$lost.log 2>&1
    tail -1 $out/pipe_${lib}_${shape//,/_}_l$lost.log
  done
done
