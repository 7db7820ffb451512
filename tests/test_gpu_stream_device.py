"""xec_decode on a stream of another device than the current one (ADVICE r3,
medium): the library buffers, copy stream and staging a decode uses are the
stream's device's, and the caller's current device is left as it was.

Needs two GPUs (skipped on the one-GPU box; the driver's 8-GPU node runs it).
The one-GPU case -- the stream's device IS the current one -- is every other
decode test."""
from __future__ import annotations

import numpy as np
import pytest

import xorec_oracle as xo

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tiling", [0, 1, 3])
def test_decode_on_other_devices_stream(gpu, tiling):
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    xec = gpu
    S, k, m, bs = 64, 16, 1, 65536
    assert xec.init(1) == 0
    torch.cuda.set_device(1)
    s1 = torch.cuda.Stream(device=1)
    d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda:1")
    p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda:1")
    assert xec.fill_splitmix64(d, S, k * bs, xo.RANDOM_SEED, s1) == 0
    assert xec.encode(d, p, S, bs, k, m, s1) == 0
    s1.synchronize()
    want = d.cpu()
    bm = xo.single_erasure_bitmap(S, k, m)
    h_bm = torch.from_numpy(bm).pin_memory()
    d_bm = h_bm.to("cuda:1")
    assert xec.erase(d, p, S, bs, k, m, d_bm, s1) == 0
    # keep s1 busy so the side-upload path (library buffers) is the one taken
    busy = torch.empty(1 << 28, dtype=torch.uint8, device="cuda:1")
    with torch.cuda.stream(s1):
        busy.fill_(1)
    torch.cuda.set_device(0)  # the current device is NOT the stream's
    assert xec.set_decode_tiling(tiling) == 0
    try:
        assert xec.decode(d, p, S, bs, k, m, h_bm, torch.empty_like(d_bm), s1) == 0
    finally:
        assert xec.set_decode_tiling(0) == 0
    assert torch.cuda.current_device() == 0
    s1.synchronize()
    assert np.array_equal(d.cpu().numpy(), want.numpy())
