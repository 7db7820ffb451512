#!/bin/bash
# where does 32+4 x 1 MiB lose against the roofline?
# read-only ceilings by geometry (tools/lab/read_probe.hip), HIP-event rates by
# loss pattern, then rocprofv3 timed-launch stats and PMC HBM bytes of the
# encode and of the reference-style (select_lost_blocks) and one-random-block
# decodes (tools/lab/shape_profile.py).  Output: gpurun_out/r05d/.
set -euo pipefail
O=gpurun_out/r05d
mkdir -p $O
export TMPDIR=/tmp
python3 -c "import sys; sys.path.insert(0, 'erasure-code-benchmark_amd'); import xec; print(xec.build_info())" > $O/build_info.txt
timeout -k 10 240 tools/lab/read_probe $O/read_probe.json > $O/read_probe.log 2>&1
for SH in 32,4,1048576,256 16,2,1048576,256; do
  for P in select random1 same rotating; do
    timeout -k 10 120 python3 tools/lab/shape_profile.py --shape $SH --pattern $P >> $O/events.log 2>&1
  done
done
for P in select random1; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt_$P -o kt --output-format csv \
    -- python3 tools/lab/shape_profile.py --pattern $P > $O/kt_$P.log 2>&1
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $O/pmc_${P}_$C -o pmc --output-format csv \
      -- python3 tools/lab/shape_profile.py --pattern $P --iters 5 > $O/pmc_${P}_$C.log 2>&1
  done
done
echo "r05d done"
