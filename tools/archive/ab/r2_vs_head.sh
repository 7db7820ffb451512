# Round-2 final library (b62decc) against the tree, in one process.
set -e
out=gpurun_out/${1:-r03m}
mkdir -p $out
for w in cfg3 cfg2 cfg4 16,8,65536,16384; do
  timeout -k 10 240 python -u tools/ab/ab.py --libs r2final,head --workload $w --rounds 9 --iters 10 \
    --out $out/r2_vs_head_${w//,/_}.json
done
