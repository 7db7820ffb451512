"""Randomised shapes and launch shapes against the oracle (seeded, bit-exact),
plus the block-size extreme where the kernels leave the 32-bit buffer-offset
store path (bs > 2 GiB, xec_api.cpp launch_shape)."""
from __future__ import annotations

import os

import numpy as np
import pytest

from test_gpu_parity import encode_and_check, erase_decode_check

pytestmark = pytest.mark.gpu

# Case counts and a seed offset for longer runs on the GPU box (defaults are the
# suite's): XEC_FUZZ_CASES=400 XEC_FUZZ_SEED=10000 pytest tests/test_gpu_fuzz.py -m gpu
N_SHAPE_CASES = int(os.environ.get("XEC_FUZZ_CASES", "48"))
N_PATH_CASES = int(os.environ.get("XEC_FUZZ_CASES", "24"))
SEED_OFFSET = int(os.environ.get("XEC_FUZZ_SEED", "0"))

LAUNCH_SHAPES = [(0, 0, 0, 0), (1, 0, 1, 64), (2, 0, 1, 64), (1, 0, 2, 256), (2, 4096, 1, 256),
                 (1, 777, 2, 64)]


def _random_case(rng):
    m = int(rng.integers(1, 9))
    k = m * int(rng.integers(1, 41))
    bs = 256 * int(rng.integers(1, 21))
    S = min(int(rng.integers(1, 10)), max(1, (24 << 20) // (k * bs)))  # oracle stays fast
    return S, k, m, bs


@pytest.mark.parametrize("case", range(N_SHAPE_CASES))
def test_random_shape_and_launch_shape(gpu, oracle, case):
    case += SEED_OFFSET
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


DECODE_PATHS = ["auto", "stripe", "class", "list", "mask", "per_stripe", "device", "device_list"]


def _recoverable_rows(bm, k, m):
    """is_recoverable per stripe (xorec_utils.hpp:160-175): every class has at
    most one lost block among its data members and its parity."""
    lost = bm == 0
    ok = np.ones(bm.shape[0], bool)
    for j in range(m):
        ok &= (lost[:, j:k:m].sum(axis=1) + lost[:, k + j]) <= 1
    return ok


def _decode_via(gpu, path, b, h_bm, d_bm):
    """Run one decode entry point (or forced tiling); returns the status the
    host sees (device paths: the device verdict)."""
    import torch
    S, k, m, bs = b.S, b.k, b.m, b.bs
    if path in ("auto", "stripe", "class", "list", "mask"):
        tiling = {"auto": 0, "stripe": 1, "class": 2, "list": 3, "mask": 4}[path]
        assert gpu.set_decode_tiling(tiling) == 0
        return int(gpu.decode(b.d, b.p, S, bs, k, m, h_bm, torch.empty_like(d_bm), b.stream))
    if path == "per_stripe":
        return int(gpu.decode_per_stripe(b.d, b.p, S, bs, k, m, h_bm, torch.empty_like(d_bm),
                                         None, b.stream))
    st = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    if path == "device":
        assert gpu.decode_device(b.d, b.p, S, bs, k, m, d_bm, st, b.stream) == 0
    else:
        n = gpu.device_list_bytes(S, k, m)
        w = torch.empty((n + 3) // 4, dtype=torch.int32, device="cuda")
        rc = gpu.decode_device_list(b.d, b.p, S, bs, k, m, d_bm, w, n, st, b.stream)
        if rc != 0:
            return int(rc)
    torch.cuda.synchronize()
    return int(st.item())


@pytest.mark.parametrize("case", range(N_PATH_CASES))
def test_random_shape_every_decode_path(gpu, oracle, case):
    """Every decode entry point and forced tiling on the same random shape and
    loss pattern, under a per-case column rotation, bit-exact against the oracle: the batch paths all-or-nothing
    (xorec_gpu_cmp.cu:75-81), xec_decode_per_stripe stripe by stripe
    (xorec_bm.cpp:43-58); parity never written.  k > 256 (the list's limit):
    the list-only entry points must refuse with InvalidSize and touch nothing."""
    import torch
    case += SEED_OFFSET
    rng = np.random.default_rng(777 + case)
    S, k, m, bs = _random_case(rng)
    S = max(S, 3)
    S = min(S, max(1, (24 << 20) // (k * bs)))
    # every case under a column rotation too (xec_set_rotation), encode included
    assert gpu.set_rotation([0, -1, 1, 3, 129][case % 5]) == gpu.Status.SUCCESS
    try:
        b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs, seed=1300 + case)
    finally:
        gpu.set_rotation(0)
    assert gpu.set_rotation([0, -1, 1, 3, 129][case % 5]) == gpu.Status.SUCCESS
    bm = np.ones((S, k + m), np.uint8)
    for c in range(S):
        oracle.select_lost_blocks(k, m, int(rng.integers(0, m + 1)), bm[c], 31 * case + c)
    if case % 3 == 0:  # one unrecoverable stripe
        c = int(rng.integers(0, S))
        bm[c, :] = 1
        bm[c, 0] = 0
        bm[c, k] = 0
    rec = _recoverable_rows(bm, k, m)
    h_bm = torch.from_numpy(bm.reshape(-1).copy()).pin_memory()
    d_bm = h_bm.to("cuda")
    ref_dt = torch.from_numpy(ref_d).to("cuda")
    want_p = ref_p.reshape(S, m, bs).copy()
    want_p[bm[:, k:] == 0] = 0
    try:
        for path in DECODE_PATHS:
            b.d[: S * k * bs].copy_(ref_dt)
            assert gpu.erase(b.d, b.p, S, bs, k, m, d_bm, b.stream) == 0
            erased = b.data().reshape(S, k, bs).copy()
            st = _decode_via(gpu, path, b, h_bm, d_bm)
            got = b.data().reshape(S, k, bs)
            assert np.array_equal(b.parity().reshape(S, m, bs), want_p), (path, "parity written")
            if k > 256 and path in ("per_stripe", "device_list"):
                assert st == gpu.Status.INVALID_SIZE, path
                assert np.array_equal(got, erased), path
                continue
            if path == "per_stripe":
                want = np.where(rec[:, None, None], ref_d.reshape(S, k, bs), erased)
                assert st == (0 if rec.all() else 4), path
            elif rec.all():
                want = ref_d.reshape(S, k, bs)
                assert st == 0, path
            else:
                want = erased
                assert st == 4, path
            assert np.array_equal(got, want), (path, S, k, m, bs)
    finally:
        gpu.set_decode_tiling(0)
        gpu.set_rotation(0)


@pytest.mark.parametrize("S,k,m,bs", [(3, 1000, 1, 256), (2, 512, 2, 512), (3, 264, 8, 256),
                                      (5, 1, 1, 256), (4, 2, 2, 768)])
def test_wide_and_narrow_stripes_every_decode_path(gpu, oracle, S, k, m, bs):
    """Stripes far wider than any BASELINE shape (k up to 1,000: the generic
    member loop, past the work list's k <= 256) and the narrowest (k = m): the
    reference puts no bound on k (xorec_utils.hpp:61-86 checks only k >= 1,
    m >= 1, k % m == 0).  Every stripe loses one block per class; every decode
    entry point rebuilds it bit-exactly, or refuses with InvalidSize where
    its list cannot name the block (k > 256), touching nothing."""
    import torch
    b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs, seed=5100 + k)
    bm = np.ones((S, k + m), np.uint8)
    for c in range(S):
        oracle.select_lost_blocks(k, m, m, bm[c], 61 * k + c)
        bm[c, k:] = 1  # data losses only: one per class
        if not (bm[c, :k] == 0).any():
            bm[c, c % k] = 0
    h_bm = torch.from_numpy(bm.reshape(-1).copy()).pin_memory()
    d_bm = h_bm.to("cuda")
    ref_dt = torch.from_numpy(ref_d).to("cuda")
    try:
        for path in DECODE_PATHS:
            b.d[: S * k * bs].copy_(ref_dt)
            assert gpu.erase(b.d, b.p, S, bs, k, m, d_bm, b.stream) == 0
            erased = b.data().copy()
            st = _decode_via(gpu, path, b, h_bm, d_bm)
            assert np.array_equal(b.parity(), ref_p), (path, "parity written")
            if k > 256 and path in ("per_stripe", "device_list"):
                assert st == gpu.Status.INVALID_SIZE and np.array_equal(b.data(), erased), path
                continue
            assert st == 0, (path, st)
            assert np.array_equal(b.data(), ref_d), (path, S, k, m, bs)
    finally:
        gpu.set_decode_tiling(0)


@pytest.mark.parametrize("extra", [0, 1])
def test_stripe_count_at_the_work_list_limit(gpu, extra):
    """S = 2^24 stripes is the most a work-list entry (stripe << 8 | block,
    xec_internal.h) can name; one more and xec_decode must take the bitmap
    tiles, xec_decode_per_stripe must refuse.  k=2+1, 256 B blocks (8 GiB of
    data), sparse losses including the batch's last stripe.  Checked by the
    round trip erase -> decode == pristine, parity untouched (the oracle would
    take minutes at this size)."""
    import torch
    S, k, m, bs = (1 << 24) + extra, 2, 1, 256
    s = torch.cuda.current_stream()
    d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
    p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
    assert gpu.fill_splitmix64(d, S, k * bs, 777, s) == 0
    assert gpu.encode(d, p, S, bs, k, m, s) == 0
    pristine, p0 = d.clone(), p.clone()
    bm = np.ones((S, k + m), np.uint8)
    lost = np.r_[np.arange(0, S, 4099), S - 1]  # ~4,100 stripes: sparse -> list wanted
    bm[lost, lost % k] = 0
    h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
    d_bm = h_bm.to("cuda")
    del bm
    assert gpu.erase(d, p, S, bs, k, m, d_bm, s) == 0
    assert gpu.decode(d, p, S, bs, k, m, h_bm, torch.empty_like(d_bm), s) == 0
    assert gpu.decode_tiling_used() == (3 if extra == 0 else 1)  # list / stripe tiles
    assert torch.equal(d, pristine) and torch.equal(p, p0)
    # the per-stripe entry point names blocks by list entry: refused past the limit
    assert gpu.erase(d, p, S, bs, k, m, d_bm, s) == 0
    st = gpu.decode_per_stripe(d, p, S, bs, k, m, h_bm, torch.empty_like(d_bm), None, s)
    if extra:
        assert st == gpu.Status.INVALID_SIZE
        assert not torch.equal(d, pristine)  # refused before touching anything
    else:
        assert st == 0 and torch.equal(d, pristine)
    assert torch.equal(p, p0)
