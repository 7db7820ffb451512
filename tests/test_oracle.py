"""Pin the CPU oracle before trusting it (CPU only).

1. SURVEY.md §8(c) known-answer parity hashes (reference build, survey session);
2. tests/golden/known_answers.json, produced by the reference's own sources
   (oracle/_ref/ref_driver, tests/golden/make_golden.py);
3. the live reference driver when it is present (this container only);
4. the C restatement against the independent numpy restatement.
"""
from __future__ import annotations

import subprocess
from pathlib import Path

import numpy as np
import pytest

import xorec_oracle as xo

from conftest import GOLDEN

SURVEY_KNOWN = {  # (k, m, bs) one stripe, state 1896
    (4, 1, 4096): "b2c6b787b51d553b",
    (8, 1, 65536): "7ed09decdded0a43",
    (16, 1, 1048576): "79b70a1259c271e6",
    (32, 1, 4096): "f4816739ea1136a6",
    (8, 4, 1024): "ff5c7b96c04c0292",
}


@pytest.mark.parametrize("shape", sorted(SURVEY_KNOWN))
def test_survey_known_answers(oracle, shape):
    k, m, bs = shape
    _, parity = oracle.batch(1, k, m, bs)
    assert f"{oracle.fnv1a64(parity):016x}" == SURVEY_KNOWN[shape]


def test_golden_encode_hashes(oracle, known_answers):
    for e in known_answers["encode"]:
        _, parity = oracle.batch(e["S"], e["k"], e["m"], e["bs"], seed_base=known_answers["seed"])
        assert f"{oracle.fnv1a64(parity):016x}" == e["parity_fnv"], e


def test_cfg1_raw_parity(oracle):
    _, parity = oracle.batch(1, 4, 1, 4096)
    ref = np.fromfile(GOLDEN / "cfg1_parity_k4_m1_4096.bin", dtype=np.uint8)
    assert np.array_equal(parity, ref)


def _erase(data, parity, bm, S, k, m, bs):
    rows = bm.reshape(S, k + m)
    d = data.reshape(S, k, bs)
    p = parity.reshape(S, m, bs)
    for c in range(S):
        for i in range(k + m):
            if rows[c, i] == 0:
                (d[c, i] if i < k else p[c, i - k])[:] = 0


def test_golden_decode(oracle, known_answers):
    for e in known_answers["decode"]:
        k, m, bs, S = e["k"], e["m"], e["bs"], e["S"]
        bm = np.fromfile(GOLDEN / "patterns" / e["pattern"], dtype=np.uint8)
        data, parity = oracle.batch(S, k, m, bs, seed_base=known_answers["seed"])
        assert f"{oracle.fnv1a64(data):016x}" == e["data_fnv_before"]
        _erase(data, parity, bm, S, k, m, bs)
        assert f"{oracle.fnv1a64(parity):016x}" == e["parity_fnv_erased"]
        codes = ""
        for c in range(S):
            codes += str(oracle.decode(data[c * k * bs:], parity[c * m * bs:], bs, k, m,
                                       bm[c * (k + m):]))
        assert codes == e["codes"], e
        assert f"{oracle.fnv1a64(data):016x}" == e["data_fnv_after"], e
        assert f"{oracle.fnv1a64(parity):016x}" == e["parity_fnv_after"], e


def test_golden_status_codes(oracle, known_answers):
    for e in known_answers["status"]:
        k, m, bs = e["k"], e["m"], e["bs"]
        data = oracle.aligned(max(k, 1) * max(bs, 256) + 128)
        par = oracle.aligned(max(m, 1) * max(bs, 256) + 128)
        bm = np.ones(max(k, 1) + max(m, 1) + 8, dtype=np.uint8)
        bm[0] = 0
        dp = data.ctypes.data + e["data_misalign"]
        pp = par.ctypes.data + e["parity_misalign"]
        assert oracle.encode(dp, pp, bs, k, m) == e["encode"], e
        assert oracle.decode(dp, pp, bs, k, m, bm) == e["decode"], e
        assert xo.np_check_args(bs, k, m, e["data_misalign"] % 64 == 0,
                                e["parity_misalign"] % 64 == 0) == e["encode"], e


def test_golden_validation_pattern(oracle, known_answers):
    for e in known_answers["validate"]:
        b = np.fromfile(GOLDEN / "patterns" / e["file"], dtype=np.uint8)
        assert oracle.validate_block(b, e["bs"]) == e["valid"]


@pytest.mark.parametrize("k,m,bs,S", [(4, 1, 4096, 3), (8, 4, 1024, 4), (6, 3, 512, 5),
                                      (5, 1, 768, 2), (2, 2, 256, 2), (32, 8, 256, 3)])
def test_c_matches_numpy_restatement(oracle, k, m, bs, S):
    data, parity = oracle.batch(S, k, m, bs)
    npdata = xo.make_data(S, k, bs)
    assert np.array_equal(data.reshape(S, k, bs), npdata)
    assert np.array_equal(parity.reshape(S, m, bs), xo.np_encode(npdata, m))
    assert f"{xo.fnv1a64(parity):016x}" == f"{oracle.fnv1a64(parity):016x}"
    # decode with reference-style random erasures, both restatements
    bm = np.ones((S, k + m), dtype=np.uint8)
    for c in range(S):
        assert oracle.select_lost_blocks(k, m, m, bm[c], c) == 0
        ref = np.ones(k + m, dtype=np.uint8)
        assert xo.np_select_lost_blocks(k, m, m, ref, c) == 0
        assert np.array_equal(ref, bm[c])
    bm = bm.reshape(-1)
    d_np = npdata.copy()
    d_np[bm.reshape(S, k + m)[:, :k] == 0] = 0x5A
    p_np = parity.reshape(S, m, bs).copy()
    assert xo.np_decode_batch_all_or_nothing(d_np, p_np, bm) == 0
    d_c = oracle.aligned(S * k * bs)
    d_c[:] = data
    rows = bm.reshape(S, k + m)
    d_c.reshape(S, k, bs)[rows[:, :k] == 0] = 0xA5  # lost content is irrelevant
    assert oracle.decode_batch_all_or_nothing(d_c, parity, S, bs, k, m, bm) == 0
    assert np.array_equal(d_c.reshape(S, k, bs), npdata)
    assert np.array_equal(d_np, npdata)


def test_recovery_predicates_match_numpy(oracle):
    rng = np.random.default_rng(7)
    for _ in range(3000):
        m = int(rng.integers(1, 6))
        k = m * int(rng.integers(1, 6))
        bm = rng.choice(np.array([0, 1, 1, 1, 2, 3], dtype=np.uint8), size=k + m)
        assert oracle.require_recovery(k, bm) == xo.np_require_recovery(k, bm)
        assert oracle.is_recoverable(k, m, bm) == xo.np_is_recoverable(k, m, bm)


def test_select_lost_blocks_contract(oracle):
    for k, m in [(8, 4), (16, 8), (32, 4), (4, 1)]:
        for lost in range(m + 1):
            for seed in range(20):
                bm = np.ones(k + m, dtype=np.uint8)
                assert oracle.select_lost_blocks(k, m, lost, bm, seed) == 0
                assert int((bm == 0).sum()) == lost
                assert oracle.is_recoverable(k, m, bm)
        assert oracle.select_lost_blocks(k, m, m + 1, np.ones(k + m, np.uint8), 0) == -1


@pytest.mark.skipif(not (xo.REF_DRIVER.exists() and Path("/root/reference/src").exists()),
                    reason="reference driver only runs where it was built")
@pytest.mark.parametrize("k,m,bs,S", [(16, 1, 65536, 8), (12, 4, 2048, 9), (24, 8, 1024, 5)])
def test_live_reference_driver(oracle, k, m, bs, S):
    out = subprocess.run([str(xo.REF_DRIVER), "dec", str(k), str(m), str(bs), str(S), "1896",
                          "3", "single7"], check=True, capture_output=True, text=True).stdout
    r = dict(line.split(" ", 1) for line in out.strip().splitlines())
    data, parity = oracle.batch(S, k, m, bs)
    assert f"{oracle.fnv1a64(parity):016x}" == r["parity_fnv"]
    bm = xo.single_erasure_bitmap(S, k, m)
    _erase(data, parity, bm, S, k, m, bs)
    assert oracle.decode_batch(data, parity, S, bs, k, m, bm) == 0
    assert f"{oracle.fnv1a64(data):016x}" == r["data_fnv_after"]
