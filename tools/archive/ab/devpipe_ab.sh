# The device-built-list decode with the software-pipelined walk
# (patches/devlist_pipelined.py: libxec_devpipe.so; with the work item
# prefetched a tile ahead, XEC_DEVPIPE_PREFETCH=1: libxec_devpipe2.so) against
# the tree's library, each in its own process with xec_decode_device (stripe
# tiles) timed beside it as the in-process reference.
set -e
out=gpurun_out/${1:-r02bt}
pats=${2:-"uniform sparse"}
libs=${3:-"tree devpipe"}
mkdir -p $out
SH=16,1,1048576,2048:32,1,4096,65536:16,8,65536,16384:16,2,1048576,256
for pat in $pats; do
  for lib in $libs; do
    if [ $lib = tree ]; then unset XEC_LIB; else export XEC_LIB=$PWD/tools/ab/libxec_$lib.so; fi
    timeout -k 10 400 python -u tools/archive/tiling_ab.py --device --shapes $SH --lost 1 --pattern $pat \
      --variants dev,devlist --rounds 5 --iters 8 --out $out/devpipe_${lib}_${pat}.json \
      > $out/devpipe_${lib}_${pat}.log 2>&1
    python3 -c "
import json,sys
for r in json.load(open('$out/devpipe_${lib}_${pat}.json')):
    print('$lib $pat', r['k'], r['m'], r['bs'], r['S'], 'devlist/dev', round(r['devlist']['median_ms']/r['dev']['median_ms'],3))"
  done
done
