# Launch-shape sweep of single-erasure decode (and encode) at small member counts.
set -e
out=gpurun_out/${1:-r02ar}
mkdir -p $out
for w in 16,8,65536,16384 16,4,65536,16384 32,8,65536,8192 16,2,1048576,256; do
  timeout -k 10 300 python -u tools/archive/sweep.py --workload $w --threads 64,256 --unroll 1,2 \
    --grid 0 --nt 1 --occ 0,8,4,2 --rounds 3 --iters 6 --out $out/sweep_${w//,/_}.json
done
