# DIAGNOSTIC run of tools/archive/ab/patches/decode_dst_diag.py builds (see there).
set -e
out=gpurun_out/${1:-r02aq}
mkdir -p $out
for w in 16,8,65536,16384 16,4,65536,16384 16,2,1048576,256 cfg3 32,8,65536,8192 4,2,1048576,512; do
  timeout -k 10 240 python -u tools/ab/ab.py --no-check --libs base,dshadow,dparity,dnostore \
    --workload $w --rounds 5 --iters 8 --out $out/dst_${w//,/_}.json
done
