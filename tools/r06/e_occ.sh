#!/bin/bash
# Round 6: residency at the reference's 8 MiB messages (VERDICT r05 item 3:
# every 8 MiB encode kernel runs at 2.2-3.3 TB/s).  Encode / decode kernel
# time from their own dispatch events, per xec_set_occupancy value, two
# passes; and the working tree's decode call against round 5's.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
for R in 1 2; do
  for SH in "8 4 1024 1024 1000 1" "32 8 1024 256 1000 1" "16 1 1024 512 1000 1" "32 1 1024 256 1000 1" "8 1 8192 128 1000 1"; do
    for OCC in 0 8 1 2 4; do
      echo "occ $OCC" >> $O/occ.log
      XEC_LAT_OCC=$OCC timeout -k 10 120 tools/latency/latency 0 $SH >> $O/occ.log 2>&1
    done
  done
done
for SH in "32 8 1024 256 2000 4" "32 8 1024 256 2000 8" "8 4 1024 1024 2000 1" "32 8 1024 256 2000 1"; do
  for R in 1 2; do
    LD_LIBRARY_PATH=$PWD/tools/ab/r5 timeout -k 10 120 tools/latency/latency 0 $SH >> $O/latency_r5.log 2>&1
    timeout -k 10 120 tools/latency/latency 0 $SH >> $O/latency_wt.log 2>&1
  done
done
echo "r06e done"
