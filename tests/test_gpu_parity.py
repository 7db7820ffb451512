"""Parity of the HIP path (libxec_hip.so on an MI355X) against the CPU oracle.

Bit-exact: parity after encode, every data block after erase+decode, parity
untouched by decode.  Sizes: every golden fixture shape (checked against the
reference-generated hashes too), the BASELINE.json configs at full size, and
edge shapes (S = 0/1, minimum block, ragged tiles, generic member counts).
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

import xorec_oracle as xo
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

SEED = xo.RANDOM_SEED


def _torch():
    import torch
    return torch


class Batch:
    """Device batch filled on the GPU with the shared splitmix64 convention."""

    def __init__(self, xec, S, k, m, bs, seed=SEED, pad=0):
        torch = _torch()
        self.S, self.k, self.m, self.bs = S, k, m, bs
        self.stream = torch.cuda.current_stream()
        self.d = torch.empty(max(S * k * bs, 1) + pad, dtype=torch.uint8, device="cuda")
        self.p = torch.full((max(S * m * bs, 1) + pad,), 0xEE, dtype=torch.uint8, device="cuda")
        if S:
            assert xec.fill_splitmix64(self.d, S, k * bs, seed, self.stream) == xec.Status.SUCCESS

    def data(self) -> np.ndarray:
        _torch().cuda.synchronize()
        return self.d[: self.S * self.k * self.bs].cpu().numpy()

    def parity(self) -> np.ndarray:
        _torch().cuda.synchronize()
        return self.p[: self.S * self.m * self.bs].cpu().numpy()


def encode_and_check(xec, oracle, S, k, m, bs, seed=SEED):
    b = Batch(xec, S, k, m, bs, seed)
    assert xec.encode(b.d, b.p, S, bs, k, m, b.stream) == xec.Status.SUCCESS
    ref_d, ref_p = oracle.batch(S, k, m, bs, seed_base=seed)
    assert np.array_equal(b.data(), ref_d), "device fill differs from oracle fill"
    assert np.array_equal(b.parity(), ref_p), f"parity mismatch {(S, k, m, bs)}"
    return b, ref_d, ref_p


def erase_decode_check(xec, b, ref_d, ref_p, bm, expect=0):
    torch = _torch()
    S, k, m, bs = b.S, b.k, b.m, b.bs
    h_bm = torch.from_numpy(np.ascontiguousarray(bm)).pin_memory()
    d_bm = h_bm.to("cuda")
    assert xec.erase(b.d, b.p, S, bs, k, m, d_bm, b.stream) == xec.Status.SUCCESS
    erased_d, erased_p = b.data(), b.parity()
    scratch = torch.empty_like(d_bm)
    st = xec.decode(b.d, b.p, S, bs, k, m, h_bm, scratch, b.stream)
    assert st == expect
    got_d, got_p = b.data(), b.parity()
    assert np.array_equal(got_p, erased_p), "decode wrote parity"
    if expect == xec.Status.SUCCESS:
        assert np.array_equal(got_d, ref_d), "recovered data mismatch"
    else:
        assert np.array_equal(got_d, erased_d), "failed decode modified data"
    # the erased parity is exactly the oracle parity with lost parity blocks zeroed
    rows = bm.reshape(S, k + m)
    want_p = ref_p.reshape(S, m, bs).copy()
    want_p[rows[:, k:] == 0] = 0
    assert np.array_equal(erased_p.reshape(S, m, bs), want_p)


# --------------------------------------------------------------------------
def test_golden_encode_fixtures(gpu, oracle, known_answers):
    """Every reference-generated known answer, through the HIP path."""
    for e in known_answers["encode"]:
        b = Batch(gpu, e["S"], e["k"], e["m"], e["bs"], known_answers["seed"])
        assert gpu.encode(b.d, b.p, e["S"], e["bs"], e["k"], e["m"], b.stream) == 0
        assert f"{oracle.fnv1a64(b.parity()):016x}" == e["parity_fnv"], e


def test_golden_cfg1_raw(gpu):
    b = Batch(gpu, 1, 4, 1, 4096)
    assert gpu.encode(b.d, b.p, 1, 4096, 4, 1, b.stream) == 0
    ref = np.fromfile(GOLDEN / "cfg1_parity_k4_m1_4096.bin", dtype=np.uint8)
    assert np.array_equal(b.parity(), ref)


def test_golden_decode_fixtures(gpu, oracle, known_answers):
    for e in known_answers["decode"]:
        k, m, bs, S = e["k"], e["m"], e["bs"], e["S"]
        bm = np.fromfile(GOLDEN / "patterns" / e["pattern"], dtype=np.uint8)
        b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs, known_answers["seed"])
        expect = gpu.Status.DECODE_FAILURE if "4" in e["codes"] else gpu.Status.SUCCESS
        erase_decode_check(gpu, b, ref_d, ref_p, bm, expect)
        if expect == gpu.Status.SUCCESS:
            assert f"{oracle.fnv1a64(b.data()):016x}" == e["data_fnv_after"]
            assert f"{oracle.fnv1a64(b.parity()):016x}" == e["parity_fnv_after"]


@pytest.mark.parametrize("S,k,m,bs", [
    (1, 4, 1, 4096),          # BASELINE config 1 shape
    (1024, 8, 1, 65536),      # config 2 (full size)
    (256, 16, 1, 1 << 20),    # config 3 (full size: 4 GiB data)
    (65536, 32, 1, 4096),     # config 4 (full size: 8 GiB data, > 4 GiB offsets)
])
def test_baseline_configs_full_size(gpu, oracle, S, k, m, bs):
    b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs)
    erase_decode_check(gpu, b, ref_d, ref_p, xo.single_erasure_bitmap(S, k, m))


@pytest.mark.parametrize("S,k,m,bs", [
    (1, 1, 1, 256), (3, 2, 2, 512), (2, 5, 1, 768), (3, 40, 8, 4352), (2, 64, 1, 256),
    (5, 6, 3, 512), (7, 12, 4, 2048), (9, 24, 8, 1024), (4, 36, 4, 4096), (3, 40, 8, 8192),
    (33, 16, 1, 8448), (17, 3, 1, 256 * 129), (5, 128, 2, 1024),
])
def test_edge_shapes_multi_erasure(gpu, oracle, S, k, m, bs):
    b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs)
    bm = np.ones((S, k + m), dtype=np.uint8)
    for c in range(S):
        oracle.select_lost_blocks(k, m, 1 + c % m, bm[c], c)
    erase_decode_check(gpu, b, ref_d, ref_p, bm.reshape(-1))


@pytest.mark.parametrize("misalign", [1, 2, 3, 5])
@pytest.mark.parametrize("S,k,m,bs", [(9, 16, 1, 4096), (7, 16, 4, 2048), (5, 10, 2, 1024)])
def test_unaligned_bitmap_scratch(gpu, oracle, misalign, S, k, m, bs):
    """The device bitmap scratch is caller-owned and may sit at any byte address."""
    torch = _torch()
    b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs)
    bm = np.ones((S, k + m), np.uint8)
    for c in range(S):
        oracle.select_lost_blocks(k, m, m, bm[c], 31 + c)
    bm = bm.reshape(-1)
    h_bm = torch.from_numpy(bm).pin_memory()
    d_bm = h_bm.to("cuda")
    assert gpu.erase(b.d, b.p, S, bs, k, m, d_bm, b.stream) == 0
    scratch = torch.full((bm.size + 16,), 0xFF, dtype=torch.uint8, device="cuda")
    assert gpu.decode(b.d, b.p, S, bs, k, m, h_bm, scratch.data_ptr() + misalign,
                      b.stream) == gpu.Status.SUCCESS
    assert np.array_equal(b.data(), ref_d)


def test_empty_batch_is_noop(gpu):
    torch = _torch()
    d = torch.empty(64, dtype=torch.uint8, device="cuda")
    assert gpu.encode(d, d, 0, 4096, 4, 1) == gpu.Status.SUCCESS
    assert gpu.decode(d, d, 0, 4096, 4, 1, np.zeros(1, np.uint8), d) == gpu.Status.SUCCESS


def test_no_loss_and_parity_only_loss_touch_nothing(gpu, oracle):
    S, k, m, bs = 8, 8, 4, 1024
    b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs)
    erase_decode_check(gpu, b, ref_d, ref_p, np.ones(S * (k + m), np.uint8))
    bm = np.ones((S, k + m), np.uint8)
    bm[:, k:] = 0
    erase_decode_check(gpu, b, ref_d, ref_p, bm.reshape(-1))


def test_argument_errors_launch_nothing(gpu):
    torch = _torch()
    d = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    p = torch.zeros(1 << 14, dtype=torch.uint8, device="cuda")
    S = gpu.Status
    assert gpu.encode(d.data_ptr() + 16, p, 1, 4096, 4, 1) == S.INVALID_ALIGNMENT
    assert gpu.encode(d, p.data_ptr() + 32, 1, 4096, 4, 1) == S.INVALID_ALIGNMENT
    assert gpu.encode(d, p, 1, 100, 4, 1) == S.INVALID_SIZE
    assert gpu.encode(d, p, 1, 4096, 6, 4) == S.INVALID_COUNTS
    assert gpu.encode(d, p, 1, 4096, 0, 1) == S.INVALID_COUNTS
    bm = np.ones(5, np.uint8)
    assert gpu.decode(d, p, 1, 320, 4, 1, bm, p) == S.INVALID_SIZE
    torch.cuda.synchronize()
    assert int(p.sum()) == 0


@pytest.mark.parametrize("threads", [64, 256])
@pytest.mark.parametrize("unroll", [1, 2])
@pytest.mark.parametrize("max_grid,nt", [(0, 2), (0, 1), (300, 2), (2048, 1), (0, 0)])
def test_launch_shapes_bit_exact(gpu, oracle, threads, unroll, max_grid, nt):
    assert gpu.set_launch(unroll, max_grid, nt, threads) == gpu.Status.SUCCESS
    try:
        for (S, k, m, bs) in [(24, 16, 1, 65536), (40, 32, 4, 4352), (9, 10, 2, 2816)]:
            b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs)
            bm = np.ones((S, k + m), np.uint8)
            for c in range(S):
                oracle.select_lost_blocks(k, m, m, bm[c], 77 + c)
            erase_decode_check(gpu, b, ref_d, ref_p, bm.reshape(-1))
    finally:
        gpu.set_launch(0, 0, 0, 0)


@pytest.mark.parametrize("threads", [64, 256])
@pytest.mark.parametrize("occ", [1, 3, 7, 8])
def test_occupancy_caps_bit_exact(gpu, oracle, threads, occ):
    """xec_set_occupancy only reserves LDS per workgroup: results stay bit-exact."""
    assert gpu.set_launch(0, 0, 0, threads) == gpu.Status.SUCCESS
    assert gpu.set_occupancy(occ) == gpu.Status.SUCCESS
    try:
        for (S, k, m, bs) in [(24, 16, 1, 65536), (40, 32, 4, 4352)]:
            b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs)
            bm = np.ones((S, k + m), np.uint8)
            for c in range(S):
                oracle.select_lost_blocks(k, m, m, bm[c], 91 + c)
            erase_decode_check(gpu, b, ref_d, ref_p, bm.reshape(-1))
    finally:
        gpu.set_occupancy(0)
        gpu.set_launch(0, 0, 0, 0)


def test_encode_is_linear(gpu):
    """Size-independent property at a full config shape: E(a ^ b) == E(a) ^ E(b)."""
    torch = _torch()
    S, k, m, bs = 256, 16, 1, 1 << 20
    a = Batch(gpu, S, k, m, bs, seed=11)
    bb = Batch(gpu, S, k, m, bs, seed=22)
    ab = torch.bitwise_xor(a.d, bb.d)
    pab = torch.empty_like(a.p)
    for x, px in ((a.d, a.p), (bb.d, bb.p), (ab, pab)):
        assert gpu.encode(x, px, S, bs, k, m, a.stream) == 0
    torch.cuda.synchronize()
    assert torch.equal(torch.bitwise_xor(a.p, bb.p), pab)


@pytest.mark.parametrize("tiling", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("S,k,m,bs,pattern", [
    (64, 16, 2, 65536, "all"),      # every class lost a data block
    (48, 16, 8, 8192, "all"),       # 8 per stripe > the 6 list entries the scratch holds: bitmap
    (64, 16, 4, 4096, "sparse"),    # a few stripes lost a block, most none
    (64, 16, 8, 2048, "skew"),      # some stripes lost a block in every class, the rest none
    (3, 264, 8, 256, "all"),        # k > 256: no work list, bitmap path
    (2048, 4, 1, 256, "one"),       # 2,048 lost blocks: past the kernel-argument list (1,024)
    (4096, 8, 4, 256, "half"),      # 8,192: a device-memory list under tiling 3
    (40, 32, 8, 4352, "all"),       # ragged tail tile
    (33, 8, 2, 2048, "all"),
    (50, 16, 4, 4096, "half"),      # half the classes: class tiles with idle tiles (auto)
    (50, 16, 4, 4096, "one"),       # one per stripe: stripe tiles (auto)
    (30, 12, 4, 1024, "parity"),    # lost parity + lost data in other classes
    (21, 24, 8, 1024, "select"),    # reference select_lost_blocks, 1..m per stripe
    (9, 10, 5, 768, "all"),         # generic member count (k/m = 2, m = 5)
    (7, 15, 5, 512, "all"),         # generic member count 3
    (16, 16, 2, 1 << 20, "device"),  # one failed device: the same data block in every stripe
    (2048, 4, 1, 256, "device"),    # the same, past the kernel-argument list
    (40, 32, 8, 4352, "devices"),   # two failed devices, in two classes
])
def test_decode_tilings_bit_exact(gpu, oracle, tiling, S, k, m, bs, pattern):
    """xec_set_decode_tiling: stripe tiles, class tiles, work-list tiles,
    kernel-argument masks and the automatic choice rebuild the same bytes, whatever fraction of the classes
    lost a block and however the losses spread over the stripes."""
    b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs)
    bm = np.ones((S, k + m), np.uint8)
    rng = np.random.default_rng(S * 1000 + k)
    for c in range(S):
        if pattern == "all":
            for j in range(m):
                bm[c, j + m * int(rng.integers(k // m))] = 0
        elif pattern == "half":
            for j in range(0, m, 2):
                bm[c, j + m * int(rng.integers(k // m))] = 0
        elif pattern == "one":
            bm[c, int(rng.integers(k))] = 0
        elif pattern == "sparse":
            if c % 9 == 4:
                bm[c, int(rng.integers(k))] = 0
        elif pattern == "skew":
            if c % 5 == 0:
                for j in range(m):
                    bm[c, j + m * int(rng.integers(k // m))] = 0
        elif pattern == "device":
            bm[c, k // 3] = 0
        elif pattern == "devices":
            bm[c, 1] = 0
            bm[c, 2 * m] = 0  # class 0, while block 1 is in class 1
        elif pattern == "parity":
            lost_par = int(rng.integers(m))
            bm[c, k + lost_par] = 0
            for j in range(m):
                if j != lost_par:
                    bm[c, j + m * int(rng.integers(k // m))] = 0
        else:
            oracle.select_lost_blocks(k, m, 1 + c % m, bm[c], 300 + c)
    assert gpu.set_decode_tiling(tiling) == gpu.Status.SUCCESS
    try:
        erase_decode_check(gpu, b, ref_d, ref_p, bm.reshape(-1))
    finally:
        gpu.set_decode_tiling(0)


@pytest.mark.parametrize("rot", [-1, 0, 1, 3, 129, 1 << 20])
@pytest.mark.parametrize("S,k,m,bs,pattern,tiling", [
    (16, 16, 2, 1 << 20, "device", 0),   # one failed device at 1 MiB: automatic rotation engages
    (16, 8, 2, 1 << 20, "device", 1),    # the same on stripe tiles
    (12, 16, 4, 1 << 20, "device", 2),   # ... class tiles
    (2048, 4, 1, 256, "device", 3),      # one chunk per block: rotation is the identity
    (40, 32, 8, 4352, "all", 0),         # ragged tail chunk moved by the rotation
    (33, 8, 2, 2048 + 768, "one", 3),    # ragged, device-memory list
    (9, 10, 5, 768, "all", 0),           # generic member count, one ragged chunk
    (16, 16, 2, 1 << 20, "device", 4),   # one failed device over stripe tiles of loss masks
    (33, 8, 2, 2048 + 768, "one", 4),    # ragged, loss masks
])
def test_rotation_bit_exact(gpu, oracle, rot, S, k, m, bs, pattern, tiling):
    """xec_set_rotation: every column rotation, automatic (0) and none (-1)
    included, gives the oracle's parity and rebuilds the same bytes, on every
    decode tiling, ragged tail chunks included (round 4)."""
    assert gpu.set_rotation(rot) == gpu.Status.SUCCESS
    assert gpu.set_decode_tiling(tiling) == gpu.Status.SUCCESS
    try:
        b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs)
        bm = np.ones((S, k + m), np.uint8)
        rng = np.random.default_rng(S * 7 + k)
        for c in range(S):
            if pattern == "device":
                bm[c, k // 3] = 0
            elif pattern == "one":
                bm[c, int(rng.integers(k))] = 0
            else:
                for j in range(m):
                    bm[c, j + m * int(rng.integers(k // m))] = 0
        erase_decode_check(gpu, b, ref_d, ref_p, bm.reshape(-1))
        # the device-resident decodes under the same rotation
        torch = _torch()
        d_bm = torch.from_numpy(np.ascontiguousarray(bm.reshape(-1))).to("cuda")
        status = torch.zeros(1, dtype=torch.int32, device="cuda")
        work = torch.empty(gpu.device_list_bytes(S, k, m), dtype=torch.uint8, device="cuda")
        h_bm = torch.from_numpy(np.ascontiguousarray(bm.reshape(-1))).pin_memory()
        for call in ("per_stripe", "device", "device_list"):
            assert gpu.erase(b.d, b.p, S, bs, k, m, d_bm, b.stream) == gpu.Status.SUCCESS
            if call == "per_stripe":  # rotation from its own list's classes
                st = gpu.decode_per_stripe(b.d, b.p, S, bs, k, m, h_bm, torch.empty_like(d_bm),
                                           None, b.stream)
                status.zero_()
            elif call == "device":
                st = gpu.decode_device(b.d, b.p, S, bs, k, m, d_bm, status, b.stream)
            else:
                st = gpu.decode_device_list(b.d, b.p, S, bs, k, m, d_bm, work, work.numel(),
                                            status, b.stream)
            assert st == gpu.Status.SUCCESS
            assert int(status.item()) == 0
            assert np.array_equal(b.data(), ref_d), call
    finally:
        gpu.set_decode_tiling(0)
        gpu.set_rotation(0)


def test_rotation_argument_range(gpu):
    for bad in (-2, (1 << 20) + 1):
        assert gpu.set_rotation(bad) == gpu.Status.INVALID_SIZE
    for ok in (-1, 0, 5, 1 << 20):
        assert gpu.set_rotation(ok) == gpu.Status.SUCCESS
    assert gpu.set_rotation(0) == gpu.Status.SUCCESS


@pytest.mark.parametrize("tiling", [1, 2, 3, 4])
def test_golden_decode_fixtures_each_tiling(gpu, oracle, known_answers, tiling):
    assert gpu.set_decode_tiling(tiling) == gpu.Status.SUCCESS
    try:
        test_golden_decode_fixtures(gpu, oracle, known_answers)
    finally:
        gpu.set_decode_tiling(0)


@pytest.mark.parametrize("S,k,m,bs,lost", [
    (1024, 8, 1, 1024, 1), (1024, 8, 1, 1024, 64),        # capacity 64, at its edge
    (1024, 8, 1, 1024, 65), (1024, 8, 1, 1024, 256),      # 256
    (1024, 8, 1, 1024, 257), (1024, 8, 1, 1024, 1024),    # 1024, the largest
    (300, 16, 4, 2048, 200), (300, 16, 4, 2048, 900),     # several per stripe, m = 4
    (64, 32, 1, 4352, 64),                                # ragged tail tile, 32 members
])
def test_decode_arg_list_capacities_bit_exact(gpu, oracle, S, k, m, bs, lost):
    """The kernel-argument work list ships the smallest of 64 / 256 / 1024
    entries that holds it (xec_kernels.h arg_items_capacity):
    every capacity, on both sides of each boundary, rebuilds bit-exactly."""
    b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs)
    bm = np.ones((S, k + m), np.uint8)
    rng = np.random.default_rng(S + lost)
    classes = [(c, j) for c in range(S) for j in range(m)]
    for idx in rng.choice(len(classes), size=lost, replace=False):
        c, j = classes[idx]
        bm[c, j + m * int(rng.integers(k // m))] = 0
    assert gpu.set_decode_tiling(3) == gpu.Status.SUCCESS
    try:
        erase_decode_check(gpu, b, ref_d, ref_p, bm.reshape(-1))
        assert gpu.decode_tiling_used() == 4
        want = 64 if lost <= 64 else 256 if lost <= 256 else 1024
        assert gpu.decode_arg_capacity_used() == want
    finally:
        gpu.set_decode_tiling(0)


@pytest.mark.parametrize("S,k,m,bs,per_stripe,expect", [
    (256, 32, 8, 1024, 8, 5),    # the reference's row 1126: 8 MiB, (40/32), 8 lost per stripe
    (256, 32, 8, 1024, 4, 5),    # 1,024 lost, dense: class tiles would upload the bitmap
    (64, 16, 2, 4096, 2, 5),     # capacity 64, at its edge
    (65, 16, 4, 1024, 4, 5),     # 256
    (257, 8, 2, 512, 2, 5),      # 1024
    (1024, 32, 4, 256, 4, 5),    # 1,024 stripes: the largest, k = 32
    (600, 12, 4, 768, 3, 5),     # generic member count 3, 1,800 lost
    (40, 32, 8, 4352, 8, 5),     # ragged tail tile
    (1000, 16, 8, 1024, 2, 6),   # 2,000 lost, a quarter of the classes: stripe tiles
    (700, 24, 8, 512, 3, 6),     # generic member count 3 on stripe tiles
    (1025, 8, 2, 256, 2, 2),     # one stripe past the argument masks: class tiles, uploaded
    (64, 40, 8, 256, 8, 2),      # k > 32: class tiles, uploaded
])
def test_decode_arg_masks_bit_exact(gpu, oracle, S, k, m, bs, per_stripe, expect):
    """Small batches (S <= 1,024, k <= 32) whose decode would upload the bitmap or
    a list send one loss mask per stripe in the kernel arguments instead
    (decode_argmask_kernel, over class tiles (5) or stripe tiles (6) by the
    bitmap path's rule): bit-exact at every capacity and on both sides of the
    limits, with the capacity reported as for the kernel-argument list."""
    b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs)
    bm = np.ones((S, k + m), np.uint8)
    rng = np.random.default_rng(S * 7 + k)
    for c in range(S):
        for j in rng.choice(m, size=per_stripe, replace=False):
            bm[c, j + m * int(rng.integers(k // m))] = 0
    erase_decode_check(gpu, b, ref_d, ref_p, bm.reshape(-1))
    assert gpu.decode_tiling_used() == expect
    if expect in (5, 6):
        assert gpu.decode_arg_capacity_used() == (64 if S <= 64 else 256 if S <= 256 else 1024)


@pytest.mark.parametrize("S,k,m,bs,kind,expect", [
    (100, 16, 1, 2048, "one", 6),      # m = 1: stripe tiles
    (96, 8, 2, 4096, "sparse", 6),     # sparse: stripe tiles, most of them idle
    (30, 12, 4, 1024, "parity", 5),    # lost parity beside lost data in the other classes
])
def test_decode_arg_masks_forced(gpu, oracle, S, k, m, bs, kind, expect):
    """xec_set_decode_tiling(4) takes the argument masks wherever they apply,
    also where the automatic policy would pass a list; class tiles or stripe
    tiles by the bitmap path's rule."""
    b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs)
    rng = np.random.default_rng(S + m)
    bm = np.ones((S, k + m), np.uint8)
    for c in range(S):
        if kind == "one" or (kind == "sparse" and c % 9 == 4):
            bm[c, (7 * c) % k] = 0
        else:
            lost_par = int(rng.integers(m))
            bm[c, k + lost_par] = 0
            for j in range(m):
                if j != lost_par:
                    bm[c, j + m * int(rng.integers(k // m))] = 0
    assert gpu.set_decode_tiling(4) == gpu.Status.SUCCESS
    try:
        erase_decode_check(gpu, b, ref_d, ref_p, bm.reshape(-1))
        assert gpu.decode_tiling_used() == expect
    finally:
        gpu.set_decode_tiling(0)


def test_decode_tiling_argument_range(gpu):
    assert gpu.set_decode_tiling(5) == gpu.Status.INVALID_SIZE
    assert gpu.set_decode_tiling(4) == gpu.Status.SUCCESS
    assert gpu.set_decode_tiling(-1) == gpu.Status.INVALID_SIZE
    assert gpu.set_decode_tiling(0) == gpu.Status.SUCCESS


def test_grid_beyond_hip_launch_limit(gpu):
    """More tiles than HIP accepts workgroups in one launch (gridDim.x * 64 >
    2^32 - 1): the default grid is capped and the kernels grid-stride over the
    rest.  k == m == 1 makes parity a copy of data, checked on the device."""
    torch = _torch()
    S, bs = (1 << 26) + 5, 1024  # 2^26 + 5 one-KiB tiles: 64 GiB data + 64 GiB parity
    free, _ = torch.cuda.mem_get_info()
    if free < 2 * S * bs + (8 << 30):
        pytest.skip(f"needs {2 * S * bs >> 30} GiB of free HBM")
    d = torch.empty(S * bs, dtype=torch.uint8, device="cuda")
    assert gpu.fill_splitmix64(d, S, bs, 5, torch.cuda.current_stream()) == 0
    p = torch.zeros_like(d)
    assert gpu.encode(d, p, S, bs, 1, 1, torch.cuda.current_stream()) == gpu.Status.SUCCESS
    torch.cuda.synchronize()
    assert torch.equal(d[-(1 << 20):], p[-(1 << 20):])
    assert torch.equal(d, p)
    del d, p
    torch.cuda.empty_cache()


def _pattern(kind, S, k, m, rng):
    bm = np.ones((S, k + m), np.uint8)
    for c in range(S):
        if kind == "one" or (kind == "sparse" and c % 9 == 4):
            bm[c, (7 * c) % k] = 0
        elif kind == "all":
            for j in range(m):
                bm[c, j + m * int(rng.integers(k // m))] = 0
        elif kind == "parity_only":
            bm[c, k] = 0
        elif kind == "double":
            if c == S // 2:
                bm[c, 0] = bm[c, m] = 0  # two losses in class 0: DecodeFailure
    return bm


def _valid_tilings(bm, k, m):
    """Every tiling xec_decode may launch for this bitmap (include/xec.h): stripe
    tiles always; class tiles when m > 1; device-list tiles when the list fits
    the S*(k+m)-byte scratch; kernel-argument list up to 1,024 blocks;
    kernel-argument masks up to 1,024 stripes with k <= 32."""
    lost = int((bm[:, :k] == 0).sum())
    S = bm.shape[0]
    v = {1}
    if m > 1:
        v.add(2)
    if k <= 256 and S <= (1 << 24) and lost <= (S * (k + m) - 3) // 4:
        v.add(3)
    if k <= 256 and S <= (1 << 24) and lost <= 1024:
        v.add(4)
    if S <= 1024 and k <= 32:
        v |= {5, 6}
    return v


@pytest.mark.parametrize("S,k,m,bs,kind,tiling", [
    (16, 16, 1, 65536, "one", 0),
    (1024, 8, 1, 4096, "one", 0),      # exactly 1,024 lost blocks
    (2048, 4, 1, 256, "one", 0),       # 2,048, every stripe
    (18432, 4, 1, 256, "sparse", 0),   # 2,048 lost, 1 stripe in 9
    (2048, 4, 1, 256, "sparse", 0),    # 228 lost, 1 in 9
    (64, 16, 2, 4096, "all", 0),       # every class lost a block
    (600, 8, 4, 256, "all", 0),
    (16, 16, 1, 65536, "one", 1),      # forced stripe tiles
    (64, 16, 2, 4096, "all", 2),       # forced class tiles
    (18432, 4, 1, 256, "sparse", 3),   # forced list: 2,048 entries through the scratch
    (64, 16, 2, 4096, "all", 3),       # forced list: 128 entries in the arguments
    (16, 16, 1, 65536, "parity_only", 0),  # nothing to rebuild: no launch
    (64, 8, 2, 1024, "double", 0),     # DecodeFailure: no launch
])
def test_decode_tiling_policy(gpu, oracle, S, k, m, bs, kind, tiling):
    """Whatever tiling the automatic policy picks -- its thresholds are tuning,
    not contract (DESIGN.md §3 *Decode policy margins*) -- it is one that applies
    to the batch (xec_decode_tiling_used) and rebuilds bit-exactly; a forced
    tiling is the one launched; nothing is launched when nothing is rebuilt."""
    b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs)
    bm = _pattern(kind, S, k, m, np.random.default_rng(S + k))
    assert gpu.set_decode_tiling(tiling) == gpu.Status.SUCCESS
    try:
        expect = gpu.Status.DECODE_FAILURE if kind == "double" else gpu.Status.SUCCESS
        erase_decode_check(gpu, b, ref_d, ref_p, bm.reshape(-1), expect=expect)
        used = gpu.decode_tiling_used()
        if kind in ("parity_only", "double"):
            assert used == 0
        elif tiling in (1, 2):
            assert used == tiling
        elif tiling == 3:  # work-list tiles: in the scratch, or in the arguments when short
            assert used == (4 if int((bm[:, :k] == 0).sum()) <= 1024 else 3)
        else:
            assert used in _valid_tilings(bm, k, m), used
    finally:
        gpu.set_decode_tiling(0)


def test_decode_refuses_graph_capture(gpu, oracle):
    """xec_decode scans h_bitmap on the host at call time, so a captured graph
    would replay that call's losses whatever the bitmap held later: on a stream
    being captured it returns XEC_DEVICE_ERROR with nothing queued (the capture
    stays valid), as does xec_decode_per_stripe.  xec_decode_device is the
    capturable form (tests/test_gpu_decode_device.py)."""
    torch = _torch()
    S, k, m, bs = 64, 16, 2, 4096
    b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs)
    bm = _pattern("all", S, k, m, np.random.default_rng(3)).reshape(-1)
    h_bm = torch.from_numpy(np.ascontiguousarray(bm)).pin_memory()
    scratch = torch.empty(bm.size, dtype=torch.uint8, device="cuda")
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=torch.cuda.Stream()):
        cs = torch.cuda.current_stream()
        assert gpu.decode(b.d, b.p, S, bs, k, m, h_bm, scratch, cs) == gpu.Status.DEVICE_ERROR
        assert gpu.decode_per_stripe(b.d, b.p, S, bs, k, m, h_bm, scratch, None,
                                     cs) == gpu.Status.DEVICE_ERROR
    g.replay()  # an empty graph
    torch.cuda.synchronize()
    del g
    erase_decode_check(gpu, b, ref_d, ref_p, bm)  # outside a capture: rebuilt


def test_decode_verdicts_from_the_scan_under_capture(gpu, oracle):
    """A batch with nothing to rebuild, or that cannot be rebuilt, gets its
    verdict from the host scan before any device call -- the reference's order
    (xorec_gpu_cmp.cu:75-81) -- also on a capturing stream; a batch with work
    is refused there, small bitmap or one past the copy-before-scan size
    (256 KiB), with nothing queued."""
    torch = _torch()
    S, k, m, bs = 64, 16, 2, 4096
    b, ref_d, ref_p = encode_and_check(gpu, oracle, S, k, m, bs)
    none = np.ones(S * (k + m), np.uint8)
    bad = none.reshape(S, k + m).copy()
    bad[5, 0] = bad[5, 2] = 0  # two losses in class 0: unrecoverable
    work = _pattern("all", S, k, m, np.random.default_rng(4)).reshape(-1)
    # 32,768 stripes x 10 blocks = 320 KiB of bitmap: the copy-first size
    Sb, kb, mb, bsb = 32768, 8, 2, 256
    big = Batch(gpu, Sb, kb, mb, bsb)
    assert gpu.encode(big.d, big.p, Sb, bsb, kb, mb, big.stream) == 0
    big_none = np.ones(Sb * (kb + mb), np.uint8)
    big_work = big_none.reshape(Sb, kb + mb).copy()
    big_work[:, 3] = 0
    pin = {n: torch.from_numpy(np.ascontiguousarray(x.reshape(-1))).pin_memory()
           for n, x in (("none", none), ("bad", bad), ("work", work),
                        ("big_none", big_none), ("big_work", big_work))}
    scratch = torch.empty(Sb * (kb + mb), dtype=torch.uint8, device="cuda")
    before = (b.data().copy(), big.data().copy())
    St = gpu.Status
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=torch.cuda.Stream()):
        cs = torch.cuda.current_stream()
        assert gpu.decode(b.d, b.p, S, bs, k, m, pin["none"], scratch, cs) == St.SUCCESS
        assert gpu.decode(b.d, b.p, S, bs, k, m, pin["bad"], scratch, cs) == St.DECODE_FAILURE
        assert gpu.decode(b.d, b.p, S, bs, k, m, pin["work"], scratch, cs) == St.DEVICE_ERROR
        assert gpu.decode(big.d, big.p, Sb, bsb, kb, mb, pin["big_none"], scratch,
                          cs) == St.SUCCESS
        assert gpu.decode(big.d, big.p, Sb, bsb, kb, mb, pin["big_work"], scratch,
                          cs) == St.DEVICE_ERROR
        assert gpu.decode_per_stripe(b.d, b.p, S, bs, k, m, pin["none"], scratch, None,
                                     cs) == St.SUCCESS
    g.replay()  # an empty graph: nothing was queued
    torch.cuda.synchronize()
    del g
    assert np.array_equal(b.data(), before[0]) and np.array_equal(big.data(), before[1])


def test_decode_scratch_upload_fallback():
    """The fallback path of xec_decode's uploads (the caller's scratch, on the
    stream) -- taken when no library buffer can be had, forced here with
    XEC_SCRATCH_UPLOADS=1 in a child process: bitmap tiles, a device work list
    longer than the kernel arguments hold, a list denser than the scratch, and
    xec_decode_per_stripe's pieces, all checked against the oracle
    (tests/scratch_uploads_check.py)."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, XEC_SCRATCH_UPLOADS="1")
    p = subprocess.run([sys.executable, str(Path(__file__).parent / "scratch_uploads_check.py")],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0 and "scratch uploads ok" in p.stdout, p.stdout[-3000:] + p.stderr[-3000:]


def test_golden_decode_fixtures_per_stripe(gpu, oracle, known_answers):
    """xec_decode_per_stripe reproduces the reference CPU plugin's per-stripe
    decode (xorec_bm.cpp:43-58) bit for bit, failing stripes included: the
    per-stripe codes and the data / parity hashes after decode are the ones the
    reference itself produced (tests/golden/make_golden.py)."""
    torch = _torch()
    for e in known_answers["decode"]:
        k, m, bs, S = e["k"], e["m"], e["bs"], e["S"]
        bm = np.fromfile(GOLDEN / "patterns" / e["pattern"], dtype=np.uint8)
        b, _, _ = encode_and_check(gpu, oracle, S, k, m, bs, known_answers["seed"])
        h_bm = torch.from_numpy(bm).pin_memory()
        d_bm = h_bm.to("cuda")
        assert gpu.erase(b.d, b.p, S, bs, k, m, d_bm, b.stream) == gpu.Status.SUCCESS
        codes = np.full(S, 0xAA, np.uint8)
        st = gpu.decode_per_stripe(b.d, b.p, S, bs, k, m, h_bm, torch.empty_like(d_bm), codes,
                                   b.stream)
        want = [int(x) for x in e["codes"]]
        assert codes.tolist() == want, e["mode"]
        assert st == (gpu.Status.DECODE_FAILURE if 4 in want else gpu.Status.SUCCESS), e["mode"]
        assert f"{oracle.fnv1a64(b.data()):016x}" == e["data_fnv_after"], e["mode"]
        assert f"{oracle.fnv1a64(b.parity()):016x}" == e["parity_fnv_after"], e["mode"]


@pytest.mark.parametrize("S,k,m,bs", [(4096, 4, 2, 256), (300, 16, 4, 1024), (5000, 8, 8, 256)])
def test_per_stripe_long_lists_and_failures(gpu, oracle, S, k, m, bs):
    """More rebuilt blocks than the kernel arguments carry, and than the
    scratch holds at once (k/m small: the list goes through it in pieces);
    every 7th stripe unrecoverable and left exactly as erased."""
    torch = _torch()
    b, ref_d, _ = encode_and_check(gpu, oracle, S, k, m, bs)
    rng = np.random.default_rng(S * 31 + k)
    bm = np.ones((S, k + m), np.uint8)
    for c in range(S):
        for j in range(m):
            bm[c, j + m * int(rng.integers(k // m))] = 0
        if c % 7 == 3:
            bm[c, k + int(rng.integers(m))] = 0  # data and parity of one class: DecodeFailure
    h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
    d_bm = h_bm.to("cuda")
    assert gpu.erase(b.d, b.p, S, bs, k, m, d_bm, b.stream) == gpu.Status.SUCCESS
    erased = b.data().reshape(S, k * bs).copy()
    codes = np.zeros(S, np.uint8)
    st = gpu.decode_per_stripe(b.d, b.p, S, bs, k, m, h_bm, torch.empty_like(d_bm), codes,
                               b.stream)
    assert st == gpu.Status.DECODE_FAILURE
    bad = np.arange(S) % 7 == 3
    assert (codes[bad] == 4).all() and (codes[~bad] == 0).all()
    got = b.data().reshape(S, k * bs)
    assert np.array_equal(got[~bad], ref_d.reshape(S, k * bs)[~bad])
    assert np.array_equal(got[bad], erased[bad])
    n_rebuilt = int((bm[~bad, :k] == 0).sum())
    assert n_rebuilt > 1024
    assert gpu.decode_tiling_used() == 3
