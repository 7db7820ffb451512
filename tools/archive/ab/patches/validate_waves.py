"""Candidate: the grouped validate kernel compiled for more resident waves
(amdgpu_waves_per_eu(XEC_VW, 8) at patch time): its two 128-B segments per
lane (current + prefetched window) hold ~86 VGPRs, i.e. 5 waves per SIMD."""
import os
import sys
p = sys.argv[1]
w = int(os.environ.get("XEC_VW", "8"))
s = open(p).read()
old = "__global__ __launch_bounds__(64) void wave_validate_kernel("
assert old in s
s = s.replace(old, f"__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu({w}, 8))) "
                   "void wave_validate_kernel(", 1)
open(p, "w").write(s)
