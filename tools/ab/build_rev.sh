#!/usr/bin/env bash
# Build libxec_hip.so of a git revision (or the working tree: "WT") into
# tools/ab/libxec_<name>.so for an in-process A/B with tools/ab/ab.py.
#   tools/ab/build_rev.sh <rev|WT> <name>
set -euo pipefail
rev=$1; name=$2
root=$(cd "$(dirname "$0")/../.." && pwd)
out=$root/tools/ab/libxec_$name.so
if [ "$rev" = WT ]; then
  make -C "$root/erasure-code-benchmark_amd" xec/libxec_hip.so >/dev/null
  cp "$root/erasure-code-benchmark_amd/xec/libxec_hip.so" "$out"
else
  tmp=$(mktemp -d)
  trap 'rm -rf "$tmp"' EXIT
  git -C "$root" archive "$rev" erasure-code-benchmark_amd include | tar -x -C "$tmp"
  make -C "$tmp/erasure-code-benchmark_amd" -j8 xec/libxec_hip.so >/dev/null
  cp "$tmp/erasure-code-benchmark_amd/xec/libxec_hip.so" "$out"
fi
echo "$out"
