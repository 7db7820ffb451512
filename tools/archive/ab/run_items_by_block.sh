set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
run() { n=$1; shift; timeout -k 10 180 python3 -u tools/ab/ab.py --libs base,bysort "$@" --out $O/$n.json > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }; tail -2 $O/$n.log; }
run cfg3_rot --workload cfg3 --pattern rotating
run cfg3_rand --workload cfg3 --pattern random
run cfg3_same --workload cfg3 --pattern same
run cfg2_rot --workload cfg2 --pattern rotating
run k16m2_rand --workload 16,2,1048576,256 --pattern random
run k16m2_rot --workload 16,2,1048576,256 --pattern rotating
run k8m2_rand --workload 8,2,1048576,256 --pattern random
run cfg3_rot2 --workload cfg3 --pattern rotating
