#!/bin/bash
# classes-innermost tile order (tools/archive/ab/patches/class_inner.py) against the
# product, in one process per shape: encode, single-erasure decode (automatic
# tiling) and, at every class lost, class-tile decode.
# Usage (inside gpurun): bash tools/archive/ab/class_inner_ab.sh <out-dir>
set -euo pipefail
o=${1:?out dir}; mkdir -p "$o"
for w in 16,2,1048576,256 8,2,1048576,256 16,4,1048576,256 32,4,1048576,256 16,2,4194304,64 \
         16,4,65536,16384 16,8,65536,16384 32,8,65536,8192 16,4,4096,65536 32,8,4096,32768 cfg3; do
  timeout -k 10 240 python -u tools/ab/ab.py --libs base,classinner --workload $w --rounds 5 \
    --iters 8 --out "$o/ci_${w//,/_}.json"
done
for w in 16,2,1048576,256:2 16,4,1048576,256:4 16,8,65536,16384:8 32,8,65536,8192:8; do
  W=${w%%:*}; L=${w##*:}
  timeout -k 10 240 python -u tools/ab/ab.py --libs base,classinner --workload $W --lost $L \
    --tiling 2 --rounds 5 --iters 8 --out "$o/ci_${W//,/_}_lost$L.json"
done
