# Residency sweep of the m > 1 single-erasure decodes (xec_set_occupancy in one
# process, tools/ab/ab.py --occ): 16+2 x 1 MiB (the shape at 0.93 of its own
# read/write ceiling) and 8+2 x 1 MiB, 16+4 x 64 KiB for comparison.
set -e
out=gpurun_out/${1:-r03zo}
mkdir -p $out
for w in 16,2,1048576,256 8,2,1048576,256 16,4,65536,16384; do
  timeout -k 10 300 python -u tools/ab/ab.py --libs head --occ 0,2,3,4,6,8 --workload $w --rounds 5 --iters 8 \
    --out $out/occ_${w//,/_}.json 2>/dev/null | grep -v amdgpu
done
