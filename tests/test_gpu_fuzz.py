"""Randomised shapes and launch shapes against the oracle (seeded, bit-exact),
plus the block-size extreme where the kernels leave the 32-bit buffer-offset
store path (bs > 2 GiB, xec_api.cpp launch_shape)."""
from __future__ import annotations

import numpy as np
import pytest

from test_gpu_parity import encode_and_check, erase_decode_check

pytestmark = pytest.mark.gpu

LAUNCH_SHAPES = [(0, 0, 0, 0), (1, 0, 1, 64), (2, 0, 1, 64), (1, 0, 2, 256), (2, 4096, 1, 256),
                 (1, 777, 2, 64)]


def _random_case(rng):
    m = int(rng.integers(1, 9))
    k = m * int(rng.integers(1, 41))
    bs = 256 * int(rng.integers(1, 21))
    S = min(int(rng.integers(1, 10)), max(1, (24 << 20) // (k * bs)))  # oracle stays fast
    return S, k, m, bs


@pytest.mark.parametrize("case", range(48))
def test_random_shape_and_launch_shape(gpu, oracle, case):
    rng = np.random.default_rng(4242 + case)
    S, k, m, bs = _random_case(rng)
    shape = LAUNCH_SHAPES[case % len(LAUNCH_SHAPES)]
    assert gpu.set_launch(*shape) == gpu.Status.SUCCESS
    try:
        b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs, seed=900 + case)
        bm = np.ones((S, k + m), np.uint8)
        for c in range(S):
            lost = int(rng.integers(0, m + 1))
            oracle.select_lost_blocks(k, m, lost, bm[c], 17 * case + c)
        if case % 5 == 0:  # make one stripe unrecoverable: the whole batch must fail untouched
            c = int(rng.integers(0, S))
            bm[c, :] = 1
            bm[c, 0] = 0
            bm[c, k] = 0  # data 0 and its class parity
            erase_decode_check(gpu, b, ref_d, ref_p, bm.reshape(-1), gpu.Status.DECODE_FAILURE)
        else:
            erase_decode_check(gpu, b, ref_d, ref_p, bm.reshape(-1))
    finally:
        gpu.set_launch(0, 0, 0, 0)


def test_block_larger_than_2gib(gpu):
    """bs = 2 GiB + 256: past the buffer-store offset range, so the library
    switches to 64-bit-addressed stores.  Checked on the device: parity ==
    d0 ^ d1, and a lost d1 is rebuilt bit-exact."""
    import torch
    bs = (1 << 31) + 256
    S, k, m = 1, 2, 1
    s = torch.cuda.current_stream()
    d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
    p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
    assert gpu.fill_splitmix64(d, S, k * bs, 31337, s) == 0
    assert gpu.encode(d, p, S, bs, k, m, s) == gpu.Status.SUCCESS
    want = torch.bitwise_xor(d[:bs], d[bs:])
    assert torch.equal(p, want)
    del want
    keep = d[bs:].clone()
    bm = np.array([1, 0, 1], np.uint8)
    h_bm = torch.from_numpy(bm).pin_memory()
    d_bm = h_bm.to("cuda")
    assert gpu.erase(d, p, S, bs, k, m, d_bm, s) == 0
    assert int(d[bs:bs + 4096].count_nonzero()) == 0
    assert gpu.decode(d, p, S, bs, k, m, h_bm, torch.empty_like(d_bm), s) == gpu.Status.SUCCESS
    torch.cuda.synchronize()
    assert torch.equal(d[bs:], keep)
