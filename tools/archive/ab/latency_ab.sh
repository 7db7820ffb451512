# Per-call latency (tools/latency/latency.cpp, default sync mode) with the
# round-2 final library and the tree's, alternated twice, at the reference's
# 8 MiB rows (k=32+8, 1 KiB blocks, 256 stripes) and k=8+4 x 1 KiB x 1024.
set -e
out=gpurun_out/${1:-r03zn}
mkdir -p $out
for rep in 1 2; do
  for lib in r2 head; do
    if [ $lib = r2 ]; then export LD_LIBRARY_PATH=$PWD/tools/ab/r2lib; else unset LD_LIBRARY_PATH; fi
    for shape in "32 8 1024 256" "8 4 1024 1024"; do
      echo "== $lib $rep $shape"
      timeout -k 10 120 tools/latency/latency 0 $shape 2000 | tee -a $out/latency_${lib}_$rep.txt
    done
  done
done
