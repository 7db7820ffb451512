# The reference's own GPU rows (tools/reference_compare.py: the plugin under the
# BM_generic-equivalent loop, per-call wall clock incl. the synchronise) with
# the round-2 final library and with the tree's, alternated twice.
set -e
out=gpurun_out/${1:-r03zk}
mkdir -p $out
for rep in 1 2; do
  for lib in r2 head; do
    if [ $lib = r2 ]; then export LD_LIBRARY_PATH=$PWD/tools/ab/r2lib; else unset LD_LIBRARY_PATH; fi
    timeout -k 10 400 python -u tools/reference_compare.py --iters 50 --warmup 10 \
      --out $out/rows_${lib}_$rep.json > $out/rows_${lib}_$rep.log 2>&1
    tail -n 2 $out/rows_${lib}_$rep.log
  done
done
