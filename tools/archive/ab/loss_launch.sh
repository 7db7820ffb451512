# Decode launch shapes by loss pattern, in one process per (shape, pattern):
# the default (one-wave workgroups, 1 KiB tiles, automatic residency) against
# 2 KiB tiles per wave (unroll 2) and 256-thread workgroups at capped
# residency.  Patterns: same (block 0 in every stripe: one failed device),
# rotating (bench.py's), random.
set -e
out=gpurun_out/${1:-r03zv}
mkdir -p $out
V="0,0,0;2,64,1;2,64,2;2,64,4;1,256,2;1,256,4"
for w in 16,2,1048576,256 8,2,1048576,256 16,4,1048576,128 16,8,1048576,256 16,2,262144,1024 16,1,1048576,256; do
  for pat in same rotating random; do
    echo "== $w $pat"
    timeout -k 10 200 python -u tools/ab/ab.py --libs head --variants "$V" --workload $w --pattern $pat \
      --rounds 4 --iters 8 --out $out/ll_${pat}_${w//,/_}.json 2>/dev/null | grep -v amdgpu
  done
done
