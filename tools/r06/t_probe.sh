#!/bin/bash
# Small-kernel latency split (tools/latency probes): dispatch-timed empty / load /
# store / copy kernels at grids of 1 and of the batch's 1 KiB tiles, beside the
# codec's own kernels; the copy probe launched plainly with and without an LDS
# reservation, + stream sync, beside xec_encode + stream sync; at two of the
# reference's 8 MiB shapes (32+4 also with the residency cap off) and config 3.
# Output: gpurun_out/$1/.
set -euo pipefail
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 120 tools/latency/latency 0 8 4 1024 1024 500 > $O/probe_8_4.log 2>&1
timeout -k 10 120 tools/latency/latency 0 32 4 1024 256 500 > $O/probe_32_4.log 2>&1
XEC_LAT_OCC=8 timeout -k 10 120 tools/latency/latency 0 32 4 1024 256 500 > $O/probe_32_4_occ8.log 2>&1
timeout -k 10 120 tools/latency/latency 0 16 1 1048576 256 200 > $O/probe_cfg3.log 2>&1
grep -h "sync\|call only\|dispatch" $O/probe_8_4.log $O/probe_32_4.log $O/probe_32_4_occ8.log
