# Round-1 final library (9e07419) against the tree, in one process.
set -e
out=gpurun_out/${1:-r02bc}
mkdir -p $out
for w in cfg3 cfg2 cfg4; do
  timeout -k 10 240 python -u tools/ab/ab.py --libs r1final,head --workload $w --rounds 9 --iters 10 \
    --out $out/r1_vs_head_$w.json
done
