# Per-call latency (tools/latency/latency.cpp) of three libraries alternated
# twice: round 2's final, the tree before the capture query moved behind the
# host scan (precap), and the tree's -- at the reference's 8 MiB rows and a
# 128 MiB k=16+4 x 64 KiB batch; the no-loss decode rows are the ones the
# capture query was in front of.
set -e
out=gpurun_out/${1:-r03zz}
mkdir -p $out
for rep in 1 2; do
  for lib in r2 precap head; do
    case $lib in
      r2) export LD_LIBRARY_PATH=$PWD/tools/ab/r2lib ;;
      precap) export LD_LIBRARY_PATH=$PWD/tools/ab/precaplib ;;
      head) unset LD_LIBRARY_PATH ;;
    esac
    for shape in "32 8 1024 256" "16 4 65536 128"; do
      echo "== $lib $rep $shape"
      timeout -k 10 120 tools/latency/latency 0 $shape 2000 | tee -a $out/latency_${lib}_$rep.txt
    done
  done
done
