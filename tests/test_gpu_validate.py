"""Device-side validation payload (xec_write_validation_pattern / xec_validate_blocks)
against the oracle's restatement of utils.cpp:35-97, which the reference's own
validate_block accepts (tests/golden/known_answers.json "validate")."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[0, 1, 2], ids=["auto", "lane", "wave"])
def vmode(request, gpu):
    """xec_set_validate_kernel: automatic, lane per block, wave per block."""
    assert gpu.set_validate_kernel(request.param) == gpu.Status.SUCCESS
    yield request.param
    gpu.set_validate_kernel(0)


@pytest.mark.parametrize("nblocks,bs", [(7, 8), (5, 15), (9, 16), (4, 100), (33, 256),
                                        (64, 4096), (3, 1 << 20), (2, 4352), (5, 512),
                                        (3, 8448), (2, 8192 + 128), (3, 16640), (9, 384),
                                        (33, 1024), (5, 2048), (130, 4096)])
def test_pattern_matches_oracle_and_validates(gpu, oracle, vmode, nblocks, bs):
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


def _host_blocks_with_carries(nblocks, bs, seed):
    """Random blocks whose checksum chain carries out of 32 bits inside the
    wave kernel's segments (lanes 0 -- the segment that also holds the header
    --, 5 and 62 of window 0, lane 30 of the last), headers set to the
    reference checksum: the wave split must take its lane-after-lane fallback
    there and still agree (tests/crc_model.py)."""
    from crc_model import SEG, serial_crc, steer_to_carry
    rng = np.random.default_rng(seed)
    out = np.empty((nblocks, bs), np.uint8)
    for b in range(nblocks):
        blk = bytearray(rng.integers(0, 256, bs, dtype=np.uint8).tobytes())
        lanes = [0, 5, 62]
        last = ((bs - 1) // (64 * SEG)) * 64 * SEG
        pos = [ln * SEG + 40 + 7 * b for ln in lanes] + [last + 30 * SEG + 9]
        for q in sorted(p for p in pos if p + 1 < bs):
            steer_to_carry(blk, bs, q)
        crc = serial_crc(bytes(blk), bs)
        blk[0:4] = crc.to_bytes(4, "little")
        blk[4:8] = bs.to_bytes(4, "little")
        out[b] = np.frombuffer(bytes(blk), np.uint8)
    return out


@pytest.mark.parametrize("bs", [1024, 4096, 65536])
def test_wave_split_exact_through_carries(gpu, oracle, vmode, bs):
    import torch
    host = _host_blocks_with_carries(3, bs, bs)
    for b in range(host.shape[0]):
        assert oracle.validate_block(host[b], bs)
    d = torch.from_numpy(host.reshape(-1)).to("cuda")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    assert gpu.validate_blocks(d, host.shape[0], bs, bad, s) == gpu.Status.SUCCESS
    torch.cuda.synchronize()
    assert int(bad.item()) == 0
    d[bs + (3 * bs) // 4 + 1] ^= 1  # block 1 only
    assert gpu.validate_blocks(d, host.shape[0], bs, bad, s) == gpu.Status.SUCCESS
    torch.cuda.synchronize()
    assert int(bad.item()) == 1


def test_wave_and_lane_kernels_agree_at_config3_size(gpu):
    """BASELINE config 3's data blocks (256 stripes x 16 x 1 MiB): the wave
    and lane kernels write byte-identical payloads, both validate them, and
    each flags exactly the blocks corrupted afterwards."""
    import torch
    n, bs = 256 * 16, 1 << 20
    s = torch.cuda.current_stream()
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")
    bufs = []
    for mode in (2, 1):
        assert gpu.set_validate_kernel(mode) == gpu.Status.SUCCESS
        d = torch.empty(n * bs, dtype=torch.uint8, device="cuda")
        assert gpu.write_validation_pattern(d, n, bs, 11, s) == gpu.Status.SUCCESS
        bufs.append(d)
    try:
        torch.cuda.synchronize()
        assert torch.equal(bufs[0], bufs[1])
        del bufs[1]
        d = bufs[0]
        hits = [0, 17, 1000, n - 1]
        for mode in (2, 1):
            assert gpu.set_validate_kernel(mode) == gpu.Status.SUCCESS
            assert gpu.validate_blocks(d, n, bs, bad, s) == gpu.Status.SUCCESS
            torch.cuda.synchronize()
            assert int(bad.item()) == 0, mode
        for h in hits:
            d[h * bs + 8 + (h * 7919) % (bs - 8)] ^= 0x10
        for mode in (2, 1):
            assert gpu.set_validate_kernel(mode) == gpu.Status.SUCCESS
            assert gpu.validate_blocks(d, n, bs, bad, s) == gpu.Status.SUCCESS
            torch.cuda.synchronize()
            assert int(bad.item()) == len(hits), mode
    finally:
        gpu.set_validate_kernel(0)


def test_validate_kernel_argument_range(gpu):
    assert gpu.set_validate_kernel(3) == gpu.Status.INVALID_SIZE
    assert gpu.set_validate_kernel(-1) == gpu.Status.INVALID_SIZE
    assert gpu.set_validate_kernel(0) == gpu.Status.SUCCESS
