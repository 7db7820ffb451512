"""Decodes on caller streams that are created and destroyed call after call.

The side uploads (csrc/xec_api.cpp upload_begin) reuse a library buffer once
the kernel that read it has passed.  That used to be tracked by an event
recorded on the CALLER's stream; once the caller destroyed the stream (as a
pipeline does), querying the event raised a stray HIP error that the next
launch reported as XEC_DEVICE_ERROR (tools/fuzz_big.py --pipeline, seeds 90002
/ 91002, profiles/r04s).  The event now lives on a library stream.

test_decode_on_short_lived_streams keeps the buffers cycling through many
short-lived streams, with class-tile decodes (bitmap uploaded) queued behind an
encode so the stream is busy and the side path is taken (it passes on the old
library too: a new stream there reuses the old one's memory).  The fuzz
sequence that showed the fault -- 4 failures in 6 runs on the old library,
none since -- runs as test_pipeline_fuzz_sequence_90002."""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _hip():
    return ctypes.CDLL("libamdhip64.so.7")


@pytest.mark.parametrize("rounds", [48])
def test_decode_on_short_lived_streams(gpu, rounds):
    import torch
    hip = _hip()
    # more stripes than the kernel-argument masks cover (1,024), so the bitmap is uploaded
    S, k, m, bs = 1040, 8, 2, 4096
    d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
    p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
    cur = torch.cuda.current_stream()
    assert gpu.fill_splitmix64(d, S, k * bs, 4242, cur) == 0
    assert gpu.encode(d, p, S, bs, k, m, cur) == 0
    torch.cuda.synchronize()
    ref = d.clone()
    rng = np.random.default_rng(7)
    for r in range(rounds):
        # two lost data blocks per stripe, one per class: class tiles, bitmap uploaded
        bm = np.ones((S, k + m), np.uint8)
        for c in range(S):
            for j in range(m):
                bm[c, j + m * int(rng.integers(0, k // m))] = 0
        h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
        d_bm = h_bm.to("cuda")
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        try:
            assert gpu.encode(d, p, S, bs, k, m, s.value) == 0  # keeps the stream busy
            assert gpu.erase(d, p, S, bs, k, m, d_bm, s.value) == 0
            st = gpu.decode(d, p, S, bs, k, m, h_bm, d_bm, s.value)
            assert st == gpu.Status.SUCCESS, (r, st)
            assert hip.hipStreamSynchronize(s) == 0
        finally:
            hip.hipStreamDestroy(s)
        assert torch.equal(d, ref), r
        assert gpu.decode_tiling_used() == 2  # class tiles: the bitmap went up


def test_pipeline_fuzz_sequence_90002(gpu):
    """tools/fuzz_big.py --pipeline --seed 90002 (8 cases; case 7 is k=4+2,
    4 KiB x 25,840 stripes through one slot, pageable) with every staging
    option on, in a child process: the sequence whose pipelines' destroyed
    streams left the stale events behind."""
    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, XEC_PIPELINE_STAGE_OPTS="afe")
    r = subprocess.run([sys.executable, "-u", str(root / "tools" / "fuzz_big.py"), "--pipeline",
                        "--cases", "8", "--seed", "90002"], cwd=str(root), env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert '"all_ok": true' in r.stdout
