set -o pipefail
o=gpurun_out/r03e; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/lab/mix_ceiling.py --out $o/mix_ceiling.json > $o/mix_ceiling.log 2>&1 || { tail $o/mix_ceiling.log; exit 1; }
cat $o/mix_ceiling.log | cut -c1-400
timeout -k 10 900 python -u tools/tiling_ab.py --pattern fraction --fraction 0.1,0.25,0.5,0.67,0.75,0.85,1.0 --lost 1 --rounds 4 --iters 6 --shapes 32,1,4096,65536:16,1,1048576,1024:16,8,65536,16384:8,1,65536,16384 --out $o/tiling_fraction.json > $o/tiling_fraction.log 2>&1 || { tail $o/tiling_fraction.log; exit 1; }
echo done
