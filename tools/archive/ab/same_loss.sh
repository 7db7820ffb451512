# The one-failed-device loss pattern (block 0 lost in every stripe) at m = 2 x
# 1 MiB, where it decodes ~18 % slower than bench.py's rotating pattern
# (tools/lab/loss_pattern_probe.py): residency and launch shapes on it.
set -e
out=gpurun_out/${1:-r03zu}
mkdir -p $out
for w in 16,2,1048576,256 8,2,1048576,256; do
  for pat in same rotating; do echo "== $w $pat"
    timeout -k 10 200 python -u tools/ab/ab.py --libs head --occ 0,2,4,6,8 --workload $w --pattern $pat \
      --rounds 4 --iters 8 --out $out/occ_${pat}_${w//,/_}.json 2>/dev/null | grep -v amdgpu
  done
  for l in 2,64 1,256; do echo "== $w same launch $l"
    timeout -k 10 200 python -u tools/ab/ab.py --libs head --occ 2,4,8 --workload $w --pattern same --launch $l \
      --rounds 4 --iters 8 --out $out/launch_${l/,/_}_same_${w//,/_}.json 2>/dev/null | grep -v amdgpu
  done
done
