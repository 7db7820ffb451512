# Per-call latency (tools/latency/latency.cpp) of three libraries alternated
# twice: round 2's final; the tree with the capture query behind the host scan
# but the stream-busy query asked on every decode with work (capfix); and the
# tree's, which asks it only before an upload -- at the reference's 8 MiB rows
# and a 128 MiB k=16+4 x 64 KiB batch ("call only" is the host time of one
# xec_decode).
set -e
out=gpurun_out/${1:-r03zza}
mkdir -p $out
for rep in 1 2; do
  for lib in r2 capfix head; do
    case $lib in
      r2) export LD_LIBRARY_PATH=$PWD/tools/ab/r2lib ;;
      capfix) export LD_LIBRARY_PATH=$PWD/tools/ab/capfixlib ;;
      head) unset LD_LIBRARY_PATH ;;
    esac
    for shape in "32 8 1024 256" "16 4 65536 128"; do
      echo "== $lib $rep $shape"
      timeout -k 10 120 tools/latency/latency 0 $shape 2000 | tee -a $out/latency_${lib}_$rep.txt
    done
  done
done
