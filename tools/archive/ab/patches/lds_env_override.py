"""EXPERIMENT HOOK (never product): the LDS reserved per workgroup comes from
the XEC_LDS_BYTES environment variable when set, so residency can be swept at
finer steps than whole waves per SIMD (e.g. 10 one-wave workgroups per CU =
16 KiB each).  Patches csrc/xec_api.cpp next to the kernels file given."""
import os
import sys
api = os.path.join(os.path.dirname(sys.argv[1]), "xec_api.cpp")
s = open(api).read()
old = "  ls.lds_bytes = lds_for_occupancy(w, ls.threads);"
new = """  ls.lds_bytes = lds_for_occupancy(w, ls.threads);
  if (const char* e = std::getenv("XEC_LDS_BYTES")) ls.lds_bytes = (uint32_t)std::strtoul(e, nullptr, 0);"""
assert old in s
s = s.replace(old, new, 1)
s = s.replace("#include <atomic>", "#include <atomic>\n#include <cstdlib>", 1)
open(api, "w").write(s)
