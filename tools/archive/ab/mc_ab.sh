set -e
mkdir -p gpurun_out/r02ap
for w in 16,2,1048576,256 16,4,65536,16384 16,8,65536,16384 32,8,65536,8192 8,2,1048576,256 4,2,1048576,512; do
  timeout -k 10 240 python -u tools/ab/ab.py --libs base,mc16,mc32 --workload $w --occ 0,2,4,8 --rounds 5 --iters 8 --out gpurun_out/r02ap/mc_${w//,/_}.json
done
