"""xec_decode_device: the device-resident decode (bitmap already in HBM, verdict
in a device int32, no host scan or copy) against the oracle and against the
host-bitmap xec_decode on the same inputs, plus hipGraph capture.

The batch verdict follows the reference's all-or-nothing rule
(xorec_gpu_cmp.cu:75-81, is_recoverable xorec_utils.hpp:160-175): 4 and
nothing written if any stripe lost two blocks of one class.
"""
from __future__ import annotations

import numpy as np
import pytest

import xorec_oracle as xo
from conftest import GOLDEN
from test_gpu_parity import Batch, encode_and_check

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    return torch


def _decode_dev(xec, api, d, p, S, bs, k, m, d_bm, d_status, stream, work=None):
    """One device-resident decode through `api`: "device" = xec_decode_device,
    "list" = xec_decode_device_list (scratch `work`, allocated when None)."""
    if api == "device":
        return xec.decode_device(d, p, S, bs, k, m, d_bm, d_status, stream)
    if work is None:
        work = _torch().full((xec.device_list_bytes(S, k, m) // 4,), -1, dtype=torch_int32(),
                             device="cuda")
    return xec.decode_device_list(d, p, S, bs, k, m, d_bm, work, work.numel() * 4, d_status,
                                  stream)


def torch_int32():
    return _torch().int32


APIS = ["device", "list"]


def _device_decode(xec, b, bm: np.ndarray, status_init: int = 0x7F, api: str = "device"):
    """erase per bm, then xec_decode_device (or _list); returns (verdict, data, erased data)."""
    torch = _torch()
    d_bm = torch.from_numpy(np.ascontiguousarray(bm)).to("cuda")
    d_status = torch.full((1,), status_init, dtype=torch.int32, device="cuda")
    assert xec.erase(b.d, b.p, b.S, b.bs, b.k, b.m, d_bm, b.stream) == 0
    erased = b.data()
    erased_p = b.parity()
    assert _decode_dev(xec, api, b.d, b.p, b.S, b.bs, b.k, b.m, d_bm, d_status, b.stream) == 0
    torch.cuda.synchronize()
    got_p = b.parity()
    assert np.array_equal(got_p, erased_p), "decode_device wrote parity"
    return int(d_status.item()), b.data(), erased


@pytest.mark.parametrize("api", APIS)
def test_golden_decode_fixtures_device(gpu, oracle, known_answers, api):
    for e in known_answers["decode"]:
        k, m, bs, S = e["k"], e["m"], e["bs"], e["S"]
        bm = np.fromfile(GOLDEN / "patterns" / e["pattern"], dtype=np.uint8)
        b, ref_d, _ = encode_and_check(gpu, oracle, S, k, m, bs, known_answers["seed"])
        verdict, got, erased = _device_decode(gpu, b, bm, api=api)
        if "4" in e["codes"]:
            assert verdict == gpu.Status.DECODE_FAILURE, e
            assert np.array_equal(got, erased), "failed batch was modified"
        else:
            assert verdict == gpu.Status.SUCCESS, e
            assert np.array_equal(got, ref_d), e
            assert f"{oracle.fnv1a64(got):016x}" == e["data_fnv_after"]


@pytest.mark.parametrize("api", APIS)
@pytest.mark.parametrize("k,m", [(4, 1), (16, 1), (8, 4), (12, 3), (40, 8), (6, 6), (66, 2)])
def test_random_patterns_match_oracle_and_host_decode(gpu, oracle, k, m, api):
    """Same verdict and bytes as the oracle's all-or-nothing batch decode and as
    xec_decode (host scan), on random loss patterns including unrecoverable
    ones and bitmap bytes that are neither 0 nor 1."""
    torch = _torch()
    rng = np.random.default_rng(k * 7 + m)
    bs = 1024
    for trial in range(12):
        S = int(rng.integers(1, 24))
        seed = 500 + trial
        p_loss = float(rng.choice([0.0, 0.03, 0.1, 0.25]))
        bm = (rng.random((S, k + m)) >= p_loss).astype(np.uint8)
        if trial % 3 == 0:
            bm[rng.random((S, k + m)) < 0.05] = rng.choice([2, 3, 255])
        rows = bm
        bm = np.ascontiguousarray(bm.reshape(-1))
        # oracle: erase (zero lost blocks) then all-or-nothing batch decode
        ref_d, ref_p = oracle.batch(S, k, m, bs, seed_base=seed)
        o_d, o_p = ref_d.reshape(S, k, bs).copy(), ref_p.reshape(S, m, bs).copy()
        o_d[rows[:, :k] == 0] = 0
        o_p[rows[:, k:] == 0] = 0
        od, op = oracle.aligned(o_d.size), oracle.aligned(o_p.size)
        od[:], op[:] = o_d.reshape(-1), o_p.reshape(-1)
        want = oracle.decode_batch_all_or_nothing(od, op, S, bs, k, m, bm)

        host = Batch(gpu, S, k, m, bs, seed=seed)
        dev = Batch(gpu, S, k, m, bs, seed=seed)
        assert gpu.encode(host.d, host.p, S, bs, k, m, host.stream) == 0
        assert gpu.encode(dev.d, dev.p, S, bs, k, m, dev.stream) == 0
        h_bm = torch.from_numpy(bm).pin_memory()
        d_bm = h_bm.to("cuda")
        assert gpu.erase(host.d, host.p, S, bs, k, m, d_bm, host.stream) == 0
        st_host = gpu.decode(host.d, host.p, S, bs, k, m, h_bm, torch.empty_like(d_bm),
                             host.stream)
        verdict, got, _ = _device_decode(gpu, dev, bm, api=api)
        assert verdict == want == int(st_host), (k, m, S, rows)
        assert np.array_equal(got, od), (k, m, S, rows)
        assert np.array_equal(host.data(), od)
        assert np.array_equal(dev.parity(), op)


@pytest.mark.parametrize("api", APIS)
def test_full_size_cfg3_device(gpu, api):
    """BASELINE configs[2] at full size (4 GiB): rebuilt data == a fresh fill."""
    torch = _torch()
    S, k, m, bs = 256, 16, 1, 1 << 20
    b = Batch(gpu, S, k, m, bs)
    assert gpu.encode(b.d, b.p, S, bs, k, m, b.stream) == 0
    bm = xo.single_erasure_bitmap(S, k, m)
    d_bm = torch.from_numpy(bm).to("cuda")
    d_status = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    assert gpu.erase(b.d, b.p, S, bs, k, m, d_bm, b.stream) == 0
    assert _decode_dev(gpu, api, b.d, b.p, S, bs, k, m, d_bm, d_status, b.stream) == 0
    fresh = torch.empty_like(b.d)
    assert gpu.fill_splitmix64(fresh, S, k * bs, xo.RANDOM_SEED, b.stream) == 0
    torch.cuda.synchronize()
    assert int(d_status.item()) == 0
    assert torch.equal(fresh, b.d)


@pytest.mark.parametrize("api", APIS)
def test_graph_capture_encode_erase_decode(gpu, oracle, api):
    """The device-resident path has no host work, so one hipGraph can hold
    encode -> erase -> decode; replays are bit-exact against the oracle."""
    torch = _torch()
    S, k, m, bs = 12, 8, 2, 4096
    ref_d, ref_p = oracle.batch(S, k, m, bs, seed_base=xo.RANDOM_SEED)
    b = Batch(gpu, S, k, m, bs)
    bm = np.ones((S, k + m), np.uint8)
    for c in range(S):
        oracle.select_lost_blocks(k, m, m, bm[c], 77 + c)
    d_bm = torch.from_numpy(bm.reshape(-1)).to("cuda")
    d_status = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    work = torch.full((gpu.device_list_bytes(S, k, m) // 4,), -1, dtype=torch.int32,
                      device="cuda")
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        s = torch.cuda.current_stream()
        assert gpu.encode(b.d, b.p, S, bs, k, m, s) == 0
        assert gpu.erase(b.d, b.p, S, bs, k, m, d_bm, s) == 0
        assert _decode_dev(gpu, api, b.d, b.p, S, bs, k, m, d_bm, d_status, s, work) == 0
    for _ in range(2):
        d_status.fill_(-1)
        b.d[: S * k * bs].copy_(torch.from_numpy(ref_d).to("cuda"))
        b.p.fill_(0xEE)
        g.replay()
        torch.cuda.synchronize()
        assert int(d_status.item()) == 0
        assert np.array_equal(b.data(), ref_d)
        want_p = ref_p.reshape(S, m, bs).copy()
        want_p[bm[:, k:] == 0] = 0  # erase zeroed the lost parity; decode never rebuilds it
        assert np.array_equal(b.parity().reshape(S, m, bs), want_p)


def test_device_argument_errors_and_empty_batch(gpu):
    torch = _torch()
    S_ = gpu.Status
    d = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    p = torch.zeros(1 << 14, dtype=torch.uint8, device="cuda")
    bm = torch.zeros(64, dtype=torch.uint8, device="cuda")
    st = torch.full((4,), 9, dtype=torch.int32, device="cuda")
    assert gpu.decode_device(d, p, 1, 4096, 4, 1, bm, st.data_ptr() + 2) == S_.INVALID_ALIGNMENT
    assert gpu.decode_device(d, p, 1, 4096, 4, 1, bm, 0) == S_.INVALID_ALIGNMENT
    assert gpu.decode_device(d, p, 1, 100, 4, 1, bm, st) == S_.INVALID_SIZE
    assert gpu.decode_device(d.data_ptr() + 16, p, 1, 4096, 4, 1, bm, st) == S_.INVALID_ALIGNMENT
    assert gpu.decode_device(d, p, 1, 4096, 6, 4, bm, st) == S_.INVALID_COUNTS
    assert gpu.decode_device(d, p, 1, 4096, 4, 1, 0, st) == S_.INVALID_SIZE  # null bitmap
    torch.cuda.synchronize()
    assert st.tolist() == [9, 9, 9, 9], "argument errors must enqueue nothing"
    assert gpu.decode_device(d, p, 0, 4096, 4, 1, 0, st[1:]) == S_.SUCCESS  # S=0: bitmap unused
    torch.cuda.synchronize()
    assert st.tolist() == [9, 0, 9, 9]
    st[1] = 9
    assert gpu.decode_device(d, p, 0, 4096, 4, 1, bm, st) == S_.SUCCESS
    torch.cuda.synchronize()
    assert st.tolist() == [0, 9, 9, 9]
    assert int(d.sum()) == 0 and int(p.sum()) == 0


@pytest.mark.parametrize("k,m,bs,S,every", [(16, 1, 1 << 16, 512, 9), (8, 4, 4096, 3000, 5),
                                            (32, 8, 1024, 777, 1), (40, 8, 768, 300, 3)])
@pytest.mark.parametrize("max_grid", [0, 3])
def test_device_list_sparse_patterns(gpu, k, m, bs, S, every, max_grid):
    """Only every `every`-th stripe loses blocks (1..m per stripe, one per class):
    xec_decode_device_list rebuilds exactly those, bit-exact against a fresh
    fill, with the default grid and with a 3-workgroup grid that has to walk
    the whole list (xec_set_launch max_grid)."""
    import bench
    torch = _torch()
    rng = np.random.default_rng(S + every)
    bm = np.ones((S, k + m), np.uint8)
    for c in range(0, S, every):
        lost = int(rng.integers(1, m + 1))
        bm[c:c + 1] = bench.erasure_pattern(np, 1, k, m, lost, start=c)
    b = Batch(gpu, S, k, m, bs, seed=33)
    assert gpu.encode(b.d, b.p, S, bs, k, m, b.stream) == 0
    fresh = b.data()
    assert gpu.set_launch(0, max_grid, 0, 0) == 0
    try:
        verdict, got, erased = _device_decode(gpu, b, bm.reshape(-1), api="list")
    finally:
        assert gpu.set_launch(0, 0, 0, 0) == 0
    assert verdict == 0
    assert not np.array_equal(erased, fresh)
    assert np.array_equal(got, fresh)


def test_device_list_writes_one_entry_per_lost_block(gpu):
    """The scratch after a call: count = lost data blocks, entries (after the
    header) = their (c << 8 | i) items in some order, nothing past them."""
    torch = _torch()
    S, k, m, bs = 100, 12, 4, 256
    rng = np.random.default_rng(5)
    bm = np.ones((S, k + m), np.uint8)
    want = set()
    for c in range(S):
        for j in range(m):
            if rng.random() < 0.3:
                i = j + m * int(rng.integers(0, k // m))
                bm[c, i] = 0
                want.add(c << 8 | i)
        if rng.random() < 0.2:
            bm[c, k + int(rng.integers(0, m))] = 0  # lost parity of a class: listed only if
    for c in range(S):                              # that class lost no data block
        for j in range(m):
            if bm[c, k + j] == 0 and any(bm[c, j::m][:k // m] == 0):
                bm[c, k + j] = 1
    b = Batch(gpu, S, k, m, bs)
    d_bm = torch.from_numpy(bm.reshape(-1)).to("cuda")
    st = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    n = gpu.device_list_bytes(S, k, m) // 4
    work = torch.full((n + 8,), -7, dtype=torch.int32, device="cuda")
    assert gpu.decode_device_list(b.d, b.p, S, bs, k, m, d_bm, work, (n + 8) * 4, st) == 0
    torch.cuda.synchronize()
    w = work.cpu().numpy().view(np.uint32)
    assert int(st.item()) == 0
    assert w[0] == len(want)
    hdr = n - S * m  # header words
    assert set(int(x) for x in w[hdr:hdr + len(want)]) == want
    assert (work.cpu().numpy()[hdr + len(want):] == -7).all()


def test_device_list_argument_errors(gpu):
    torch = _torch()
    S_ = gpu.Status
    d = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    p = torch.zeros(1 << 14, dtype=torch.uint8, device="cuda")
    bm = torch.zeros(64, dtype=torch.uint8, device="cuda")
    st = torch.full((4,), 9, dtype=torch.int32, device="cuda")
    w = torch.full((16,), 9, dtype=torch.int32, device="cuda")
    need = gpu.device_list_bytes(2, 4, 2)
    assert need == gpu.device_list_bytes(0, 4, 2) + 4 * 2 * 2
    call = gpu.decode_device_list
    assert call(d, p, 2, 4096, 4, 2, bm, w.data_ptr() + 2, need, st) == S_.INVALID_ALIGNMENT
    assert call(d, p, 2, 4096, 4, 2, bm, 0, need, st) == S_.INVALID_ALIGNMENT
    assert call(d, p, 2, 4096, 4, 2, bm, w, need, st.data_ptr() + 1) == S_.INVALID_ALIGNMENT
    assert call(d, p, 2, 4096, 4, 2, bm, w, need - 4, st) == S_.INVALID_SIZE
    assert call(d, p, 2, 4096, 4, 2, 0, w, need, st) == S_.INVALID_SIZE
    assert call(d, p, 1, 256, 300, 1, bm, w, 64, st) == S_.INVALID_SIZE  # k > 256
    assert call(d, p, 2, 100, 4, 2, bm, w, need, st) == S_.INVALID_SIZE
    assert call(d, p, 2, 4096, 6, 4, bm, w, need, st) == S_.INVALID_COUNTS
    torch.cuda.synchronize()
    assert st.tolist() == [9] * 4 and w.tolist() == [9] * 16, "rejected calls enqueue nothing"
    assert call(d, p, 0, 4096, 4, 2, 0, w, 0, st) == S_.SUCCESS  # S=0: verdict 0, no scratch use
    torch.cuda.synchronize()
    assert st.tolist() == [0, 9, 9, 9] and w.tolist() == [9] * 16
