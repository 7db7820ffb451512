#!/usr/bin/env bash
# Build libxec_hip.so of the working tree with a diagnostic or candidate
# source patch applied in a scratch copy (never in the tree) into
# tools/ab/libxec_<name>.so, for an in-process A/B with tools/ab/ab.py.
#   tools/ab/build_variant.sh <name> <patch.py>
# <patch.py> is run with the scratch csrc/xec_kernels.hip path as argv[1] and
# rewrites it in place.
set -euo pipefail
name=$1; patch=$2
root=$(cd "$(dirname "$0")/../.." && pwd)
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
cp -r "$root/erasure-code-benchmark_amd" "$root/include" "$tmp/"
rm -rf "$tmp/erasure-code-benchmark_amd/build" "$tmp/erasure-code-benchmark_amd/xec/"*.so
python3 "$patch" "$tmp/erasure-code-benchmark_amd/csrc/${XEC_PATCH_FILE:-xec_kernels.hip}"
make -C "$tmp/erasure-code-benchmark_amd" -j8 xec/libxec_hip.so >/dev/null
cp "$tmp/erasure-code-benchmark_amd/xec/libxec_hip.so" "$root/tools/ab/libxec_$name.so"
echo "$root/tools/ab/libxec_$name.so"
