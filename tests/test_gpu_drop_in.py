"""The drop-in plugin classes THEMSELVES on the GPU.

integration/xorec_hip_bm.cpp and integration/xorec_hip_multi_bm.cpp are the
one source of both plugins: here built into libxec_plugin.so over this repo's
restatement of the reference's interface (integration/iface/), where the
reference is mounted also against its unmodified headers
(tests/test_reference_integration.py).  tests/host/drop_in.cpp drives them
through AbstractBenchmark& as the reference's BM_generic does
(/root/reference/src/benchmark/abstract_runner.hpp:97-121) and checks each step
against the oracle: parity == oracle encode, the erasure draw recoverable (and
equal to the oracle's for a seed), decode rebuilding the pre-loss bytes
exactly with parity untouched, check_for_corruption true.
"""
from __future__ import annotations

import os
import subprocess

import pytest

from conftest import ROOT

DROP_IN = ROOT / "tests" / "host" / "bin" / "drop_in"

# (plugin, message, block, total, data, lost, seed or "-" (the reference's
# one-argument constructor: wall-clock payloads and draws), XEC_DEVICES)
CASES = [
    # BASELINE.json configs[2]: k=16+1, 1 MiB shards, 256 stripes, reference registration
    ("single", "4G", "1M", 17, 16, 1, "-", None),
    ("single", "4G", "1M", 17, 16, 1, "1896", None),
    # a reference sweep row (bm_config.cpp:3-23): (40/32), 8 MiB message, 1 KiB blocks
    ("single", "8M", "1K", 40, 32, 8, "-", None),
    ("single", "8M", "1K", 40, 32, 8, "7", None),
    # the multi-device plugin over three ranges of device 0 (XEC_DEVICES)
    ("multi", "8M", "2K", 24, 16, 4, "-", "0,0,0"),
    ("multi", "8M", "1K", 40, 32, 8, "11", "0,0,0"),
    ("multi", "512M", "1M", 17, 16, 1, "-", "0,0,0"),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(map(str, c[:7])))
def test_drop_in_plugin_bm_generic_iteration(case):
    plugin, msg, blk, tot, data, lost, seed, devices = case
    assert DROP_IN.exists(), "build with make -C tests/host"
    env = dict(os.environ)
    env.pop("XEC_DEVICES", None)
    if devices:
        env["XEC_DEVICES"] = devices
    p = subprocess.run([str(DROP_IN), plugin, msg, blk, str(tot), str(data), str(lost), seed, "2"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0 and "drop_in ok" in p.stdout, p.stdout[-3000:] + p.stderr[-3000:]
