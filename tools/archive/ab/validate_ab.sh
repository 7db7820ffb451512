# Grouped validate kernel at more resident waves (tools/archive/ab/patches/validate_waves.py)
# against the tree: tools/archive/validate_cost.py per library, alternated twice.
set -e
out=gpurun_out/${1:-r03zj}
mkdir -p $out
for rep in 1 2; do
  for lib in vbase vw6 vw8; do
    for w in cfg3 cfg2; do
      XEC_LIB=$PWD/tools/ab/libxec_$lib.so timeout -k 10 200 python -u tools/archive/validate_cost.py --workload $w \
        --out $out/validate_${lib}_${w}_$rep.json 2>/dev/null | tail -n 1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$lib $w $rep', d['auto']['validate_ms'], d['encode_ms'])"
    done
  done
done
