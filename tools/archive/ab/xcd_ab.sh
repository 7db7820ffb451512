# A/B of tools/archive/ab/patches/xcd_items.py builds (one item per XCD).
set -e
out=gpurun_out/${1:-r02as}
mkdir -p $out
for w in 16,8,65536,16384 16,4,65536,16384 32,8,65536,8192 16,2,1048576,256 cfg3 cfg2 cfg4 4,2,1048576,512; do
  timeout -k 10 240 python -u tools/ab/ab.py --libs base,xdec,xall \
    --workload $w --rounds 5 --iters 8 --out $out/xcd_${w//,/_}.json
done
