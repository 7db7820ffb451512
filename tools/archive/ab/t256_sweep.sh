# 256-thread tiles (4 KiB per member and per store) against one-wave tiles at
# the m = 1 BASELINE shapes under residency caps.
set -e
out=gpurun_out/${1:-r02au}
mkdir -p $out
for w in cfg4 cfg3 cfg2; do
  timeout -k 10 300 python -u tools/archive/sweep.py --workload $w --threads 64,256 --unroll 1 \
    --grid 0 --nt 1 --occ 0,1,2,4,8 --rounds 4 --iters 8 --out $out/t256_$w.json
done
