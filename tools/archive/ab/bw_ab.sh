# A/B of tools/archive/ab/patches/decode_block_wave.py builds at config 4.
set -e
out=gpurun_out/${1:-r02av}
mkdir -p $out
timeout -k 10 300 python -u tools/ab/ab.py --libs base,bw8,bw16,bw8e --workload cfg4 \
  --occ 0,1,2 --rounds 6 --iters 8 --out $out/bw_cfg4.json
timeout -k 10 300 python -u tools/ab/ab.py --libs base,bw8,bw8e --workload 32,1,4096,131072 \
  --rounds 5 --iters 8 --out $out/bw_32_1_4096_131072.json
