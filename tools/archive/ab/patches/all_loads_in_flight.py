"""Candidate: issue every class member's load before the first XOR (a
scheduling barrier after the load loop), instead of the compiler's rolling
window of ~11 outstanding loads.  Costs NM*4 VGPRs for the loaded granules,
which only residency-capped launches can afford."""
import sys
p = sys.argv[1]
s = open(p).read()
old = """        for (int u = 0; u < U; ++u) v[r][u] = ld16<NT>(src + u * kStep);
      }
"""
new = """        for (int u = 0; u < U; ++u) v[r][u] = ld16<NT>(src + u * kStep);
      }
      __builtin_amdgcn_sched_barrier(0);
"""
assert old in s
s = s.replace(old, new, 1)
open(p, "w").write(s)
