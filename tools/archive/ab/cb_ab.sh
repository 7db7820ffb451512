# Stores batched over CB chunks per workgroup (tools/archive/ab/patches/chunk_batch.py)
# against the tree, in one process.
set -e
out=gpurun_out/${1:-r03o}
mkdir -p $out
for w in cfg3 cfg2 cfg4; do
  timeout -k 10 240 python -u tools/ab/ab.py --libs head,cb4,cb4sb,cb2 --workload $w --rounds 9 --iters 10 \
    --out $out/cb_$w.json
done
