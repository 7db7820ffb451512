# Second box for tools/archive/ab/loss_launch.sh's candidates: 2 KiB tiles per wave at
# 1-2 waves per SIMD against the default, at 8 members per class and m >= 2
# (and 8+2 for 4 members), blocks 512 KiB - 4 MiB, three loss patterns.
set -e
out=gpurun_out/${1:-r03zw}
mkdir -p $out
V="0,0,0;2,64,1;2,64,2;1,256,2"
for w in 16,2,1048576,256 32,4,1048576,128 16,2,524288,512 16,2,4194304,64 8,2,1048576,256; do
  for pat in same rotating random; do
    echo "== $w $pat"
    timeout -k 10 200 python -u tools/ab/ab.py --libs head --variants "$V" --workload $w --pattern $pat \
      --rounds 5 --iters 8 --out $out/ll_${pat}_${w//,/_}.json 2>/dev/null | grep -v amdgpu
  done
done
