#!/usr/bin/env python3
"""Does rocprofv3 see bench.py's ROCTx calls (xec/markers.py)?  Launches 3
kernels before, 5 inside markers.timed_region("probe:timed") and 3 after;
under --marker-trace the range must appear, under --selected-regions only the
5 inner launches may be traced."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[3]
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))

import torch  # noqa: E402

from xec import markers  # noqa: E402

markers.pause()
x = torch.ones(1 << 20, device="cuda")
for _ in range(3):
    x.mul_(1.0001)
torch.cuda.synchronize()
with markers.timed_region("probe:timed"):
    for _ in range(5):
        x.add_(1.0)
    torch.cuda.synchronize()
for _ in range(3):
    x.mul_(0.9999)
torch.cuda.synchronize()
print("roctx available:", markers.available())
