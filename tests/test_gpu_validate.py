"""Device-side validation payload (xec_write_validation_pattern / xec_validate_blocks)
against the oracle's restatement of utils.cpp:35-97, which the reference's own
validate_block accepts (tests/golden/known_answers.json "validate")."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nblocks,bs", [(7, 8), (5, 15), (9, 16), (4, 100), (33, 256),
                                        (64, 4096), (3, 1 << 20), (2, 4352)])
def test_pattern_matches_oracle_and_validates(gpu, oracle, nblocks, bs):
    import torch
    seed = 77
    d = torch.empty(nblocks * bs + 16, dtype=torch.uint8, device="cuda")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    assert gpu.write_validation_pattern(d, nblocks, bs, seed, s) == gpu.Status.SUCCESS
    torch.cuda.synchronize()
    got = d[: nblocks * bs].cpu().numpy().reshape(nblocks, bs)
    for b in range(nblocks):
        want = np.zeros(bs, np.uint8)
        oracle.write_validation_pattern(want, bs, seed + b)
        assert np.array_equal(got[b], want), b
        assert oracle.validate_block(got[b], bs)
    assert gpu.validate_blocks(d, nblocks, bs, bad, s) == gpu.Status.SUCCESS
    torch.cuda.synchronize()
    assert int(bad.item()) == 0
    # corrupt a payload byte of every third block: exactly those fail
    flipped = list(range(0, nblocks, 3))
    for b in flipped:
        d[b * bs + bs - 1] ^= 0x40
    assert gpu.validate_blocks(d, nblocks, bs, bad, s) == gpu.Status.SUCCESS
    torch.cuda.synchronize()
    host = d[: nblocks * bs].cpu().numpy().reshape(nblocks, bs)
    assert int(bad.item()) == sum(not oracle.validate_block(host[b], bs) for b in range(nblocks))
    if bs >= 16:
        assert int(bad.item()) == len(flipped)


def test_pattern_survives_encode_erase_decode(gpu):
    """The reference's end-to-end check (abstract_runner.hpp:100-126) on device."""
    import torch
    S, k, m, bs = 32, 16, 4, 8192
    s = torch.cuda.current_stream()
    d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
    p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")
    assert gpu.write_validation_pattern(d, S * k, bs, 5, s) == 0
    assert gpu.encode(d, p, S, bs, k, m, s) == 0
    bm = np.ones((S, k + m), np.uint8)
    bm[:, 0] = 0
    bm[:, 5] = 0
    h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
    d_bm = h_bm.to("cuda")
    assert gpu.erase(d, p, S, bs, k, m, d_bm, s) == 0
    assert gpu.validate_blocks(d, S * k, bs, bad, s) == 0
    torch.cuda.synchronize()
    assert int(bad.item()) == 2 * S
    assert gpu.decode(d, p, S, bs, k, m, h_bm, torch.empty_like(d_bm), s) == 0
    assert gpu.validate_blocks(d, S * k, bs, bad, s) == 0
    torch.cuda.synchronize()
    assert int(bad.item()) == 0
