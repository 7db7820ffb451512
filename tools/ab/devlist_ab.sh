#!/usr/bin/env bash
# GPU box: tools/tiling_ab.py --device for the product library and the
# devlist_heads.py variants (tools/ab/libxec_<name>.so), one process each,
# uniform and sparse losses.  Every row carries the in-process xec_decode_device
# time (dev) beside devlist, so the variants compare through that ratio.
#   bash tools/ab/devlist_ab.sh <outdir> <name>...
set -euo pipefail
out=$1; shift
mkdir -p "$out"
SH=16,1,1048576,512:32,1,4096,65536:16,8,65536,16384
for lib in product "$@"; do
  for P in uniform sparse; do
    if [ "$lib" = product ]; then unset XEC_LIB; else export XEC_LIB=tools/ab/libxec_$lib.so; fi
    timeout -k 10 200 python -u tools/tiling_ab.py --device --pattern $P --shapes $SH \
      --lost 1,8 --variants list,dev,devlist --out "$out/${lib}_$P.json" > "$out/${lib}_$P.log" 2>&1
  done
done
echo done
