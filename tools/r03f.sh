set -o pipefail
o=gpurun_out/r03f; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/lab/mix_ceiling.py --out $o/mix_ceiling.json > $o/mix_ceiling.log 2>&1 || { tail $o/mix_ceiling.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $o/trace -o mt --output-format csv -- python3 tools/lab/mix_ceiling.py --shapes 16,8,65536,16384:32,8,65536,8192:32,1,4096,65536 --rounds 3 > $o/mix_traced.log 2>&1 || { tail $o/mix_traced.log; exit 1; }
find $o/trace -name '*stats*.csv' | sort
