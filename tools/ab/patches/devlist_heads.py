"""Work-queue shape of decode_devlist_kernel (xec_decode_device_list):
XEC_DL_STRIDE = u32 words between the work-queue heads, XEC_DL_GRAB = tiles
per pull (kDevListHeadStride / kDevListGrab in xec_kernels.h).  The patch
rewrites the header next to the kernels (argv[1] = scratch xec_kernels.hip)."""
import os
import re
import sys
from pathlib import Path

h = Path(sys.argv[1]).with_name("xec_kernels.h")
s = h.read_text()
for name, env in (("kDevListHeadStride", "XEC_DL_STRIDE"), ("kDevListGrab", "XEC_DL_GRAB")):
    if env in os.environ:
        s, n = re.subn(rf"(constexpr uint32_t {name} = )\d+", rf"\g<1>{int(os.environ[env])}", s)
        assert n == 1, name
h.write_text(s)
