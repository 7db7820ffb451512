# DIAGNOSTIC: work-list decode forced (--tiling 3) at the m > 1 single-erasure
# 64 KiB shapes: product vs no store / separate allocation / computed item;
# stripe tiles (--tiling 1) of the same library beside it.
set -e
out=gpurun_out/${1:-r02at}
mkdir -p $out
for w in 16,8,65536,16384 16,4,65536,16384 32,8,65536,8192 cfg4; do
  timeout -k 10 240 python -u tools/ab/ab.py --no-check --libs base,dnostore,dshadow,noitem \
    --tiling 3 --workload $w --rounds 5 --iters 8 --out $out/list_${w//,/_}.json
  timeout -k 10 240 python -u tools/ab/ab.py --libs base --tiling 1 --workload $w \
    --rounds 5 --iters 8 --out $out/stripe_${w//,/_}.json
done
