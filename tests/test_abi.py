"""The C ABI library loads, exports include/xec.h, and its host-only logic
matches the oracle (CPU only: no compute call needs a GPU here)."""
from __future__ import annotations

import re
import shutil
import subprocess

import numpy as np
import pytest

import xorec_oracle as xo
import xec
from conftest import ROOT


def header_symbols() -> set[str]:
    text = (ROOT / "include" / "xec.h").read_text()
    return set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(xec_\w+)\s*\(", text, re.M))


def test_header_and_binding_agree():
    assert header_symbols() == set(xec.EXPORTED)


def test_library_exports_every_header_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", str(xec.LIB_PATH)], check=True,
                         capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = header_symbols() - exported
    assert not missing, f"libxec_hip.so lacks {missing}"
    L = xec.lib()
    for name in header_symbols():
        assert getattr(L, name) is not None


def test_library_is_hip_gfx950(tmp_path):
    # --offloading extracts the code objects next to its input: run it on a copy
    lib = tmp_path / xec.LIB_PATH.name
    shutil.copyfile(xec.LIB_PATH, lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True, cwd=tmp_path)
    assert "gfx950" in out.stdout + out.stderr or b"gfx950" in lib.read_bytes()
    assert "gfx950" in xec.build_info()


def test_status_strings():
    names = ["Success", "InvalidSize", "InvalidAlignment", "InvalidCounts", "DecodeFailure",
             "NotInitialized", "DeviceError"]
    for code, name in enumerate(names):
        assert xec.status_string(code) == name
        assert xec.Status(code).value == code


def test_compute_before_init_is_not_initialized():
    # xec_init never succeeded in a GPU-less process, so every compute entry
    # point must refuse before touching the device (reference throws instead).
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present; covered by the process-level GPU tests")
    assert xec.init(0) == xec.Status.DEVICE_ERROR
    S, k, m, bs = 1, 4, 1, 4096
    assert xec.encode(64, 128, S, bs, k, m) == xec.Status.NOT_INITIALIZED
    bm = np.ones(5, dtype=np.uint8)
    assert xec.decode(64, 128, S, bs, k, m, bm, 256) == xec.Status.NOT_INITIALIZED
    assert xec.erase(64, 128, S, bs, k, m, 256) == xec.Status.NOT_INITIALIZED
    assert xec.fill_splitmix64(64, S, 4096, 1) == xec.Status.NOT_INITIALIZED


def test_check_args_matches_golden(known_answers):
    for e in known_answers["status"]:
        st = xec.check_args(4096 + e["data_misalign"], 8192 + e["parity_misalign"], e["bs"], e["k"],
                            e["m"])
        assert st == e["encode"], e


@pytest.mark.parametrize("bs", [0, 1, 64, 100, 255, 256, 257, 320, 512, 768, 4096, 4352,
                                1 << 20, (1 << 20) + 128])
@pytest.mark.parametrize("k,m", [(0, 1), (1, 0), (4, 1), (6, 4), (8, 4), (1, 1), (3, 2)])
def test_check_args_matches_oracle(oracle, bs, k, m):
    for da, pa in [(0, 0), (64, 0), (0, 64), (8, 0), (0, 16), (32, 48)]:
        want = oracle.check_args(4096 + da, 8192 + pa, bs, k, m)
        assert xec.check_args(4096 + da, 8192 + pa, bs, k, m) == want


def _oracle_batch_check(k, m, rows):
    need = False
    for r in rows:
        if xo.np_require_recovery(k, r):
            need = True
        if not xo.np_is_recoverable(k, m, r):
            return xo.DECODE_FAILURE, False
    return xo.SUCCESS, need


def test_check_bitmap_random(oracle):
    rng = np.random.default_rng(1896)
    for trial in range(1500):
        m = int(rng.choice([1, 2, 3, 4, 8]))
        k = m * int(rng.integers(1, 9))
        S = int(rng.integers(1, 40))
        p_loss = float(rng.choice([0.0, 0.02, 0.1, 0.3]))
        bm = (rng.random((S, k + m)) >= p_loss).astype(np.uint8)
        if trial % 5 == 0:  # values with bit 0 clear but nonzero, and odd values > 1
            bm[rng.random((S, k + m)) < 0.05] = rng.choice([2, 3, 4, 255])
        want = _oracle_batch_check(k, m, bm)
        got_st, got_need = xec.check_bitmap(bm.reshape(-1), S, k, m)
        assert int(got_st) == want[0], (k, m, S, bm)
        if want[0] == xo.SUCCESS:
            assert got_need == want[1], (k, m, S, bm)


@pytest.mark.parametrize("k,m", [(62, 2), (63, 1), (60, 4), (64, 1), (32, 32), (48, 16), (66, 2)])
def test_check_bitmap_row_width_edges(oracle, k, m):
    """Rows of 64 bytes take the per-stripe AVX2 path, wider rows the visitor;
    both must agree with the oracle, including on the last stripes, whose
    64-byte window would cross the end of the caller's buffer."""
    rng = np.random.default_rng(k * 131 + m)
    for trial in range(200):
        S = int(rng.integers(1, 12))
        p_loss = float(rng.choice([0.0, 0.01, 0.03, 0.2]))
        bm = (rng.random((S, k + m)) >= p_loss).astype(np.uint8)
        if trial % 3 == 0:
            bm[rng.random((S, k + m)) < 0.05] = rng.choice([2, 3, 254, 255])
        want = _oracle_batch_check(k, m, bm)
        got_st, got_need = xec.check_bitmap(np.ascontiguousarray(bm.reshape(-1)), S, k, m)
        assert int(got_st) == want[0], (k, m, S, bm)
        if want[0] == xo.SUCCESS:
            assert got_need == want[1], (k, m, S, bm)


def test_check_bitmap_golden_patterns(known_answers):
    from conftest import GOLDEN
    for e in known_answers["decode"]:
        k, m, S = e["k"], e["m"], e["S"]
        bm = np.fromfile(GOLDEN / "patterns" / e["pattern"], dtype=np.uint8)
        st, need = xec.check_bitmap(bm, S, k, m)
        assert (st == xec.Status.DECODE_FAILURE) == ("4" in e["codes"]), e
        if st == xec.Status.SUCCESS:
            assert need == any(xo.np_require_recovery(k, bm[c * (k + m):(c + 1) * (k + m)])
                               for c in range(S))


def test_check_bitmap_single_erasure_large():
    S, k, m = 65536, 32, 1
    bm = xo.single_erasure_bitmap(S, k, m)
    st, need = xec.check_bitmap(bm, S, k, m)
    assert st == xec.Status.SUCCESS and need
    bm2 = bm.copy()
    bm2[(S - 1) * (k + m) + k] = 0  # last stripe also loses its parity -> unrecoverable
    assert xec.check_bitmap(bm2, S, k, m)[0] == xec.Status.DECODE_FAILURE
    assert xec.check_bitmap(np.ones(S * (k + m), np.uint8), S, k, m) == (xec.Status.SUCCESS, False)


def test_set_launch_validation():
    assert xec.set_launch(3, 0, 0) == xec.Status.INVALID_SIZE
    assert xec.set_launch(4, 0, 0) == xec.Status.INVALID_SIZE
    assert xec.set_launch(1, -1, 0) == xec.Status.INVALID_SIZE
    assert xec.set_launch(1, 0, 3) == xec.Status.INVALID_SIZE
    assert xec.set_launch(1, 0, 0, 128) == xec.Status.INVALID_SIZE
    assert xec.set_launch(2, 64, 1, 256) == xec.Status.SUCCESS
    assert xec.set_launch(0, 0, 0, 0) == xec.Status.SUCCESS


def test_set_occupancy_validation():
    assert xec.set_occupancy(-1) == xec.Status.INVALID_SIZE
    assert xec.set_occupancy(9) == xec.Status.INVALID_SIZE
    for w in (1, 4, 8, 0):
        assert xec.set_occupancy(w) == xec.Status.SUCCESS


def test_tuning_snapshot_roundtrip_and_all_or_nothing():
    """xec_get_tuning / xec_set_tuning (the multi-device plugin's
    workers take the caller's overrides): a snapshot round-trips, an invalid
    field changes nothing, and another thread starts at the defaults."""
    import ctypes
    import threading
    from xec._lib import Tuning
    L = xec.lib()
    t = Tuning()
    try:
        assert xec.set_launch(2, 64, 1, 256) == xec.Status.SUCCESS
        assert xec.set_occupancy(4) == xec.Status.SUCCESS
        assert L.xec_set_decode_tiling(3) == 0 and L.xec_set_validate_kernel(1) == 0
        assert L.xec_get_tuning(ctypes.byref(t)) == 0
        assert (t.unroll, t.max_grid, t.cache_policy, t.block_threads, t.waves_per_simd,
                t.decode_tiling, t.validate_kernel) == (2, 64, 1, 256, 4, 3, 1)
        seen = {}

        def worker():
            w = Tuning()
            L.xec_get_tuning(ctypes.byref(w))
            seen["fresh"] = (w.unroll, w.decode_tiling, w.validate_kernel)
            seen["set"] = L.xec_set_tuning(ctypes.byref(t))
            L.xec_get_tuning(ctypes.byref(w))
            seen["after"] = (w.unroll, w.max_grid, w.decode_tiling, w.validate_kernel)

        th = threading.Thread(target=worker)
        th.start()
        th.join()
        assert seen == {"fresh": (0, 0, 0), "set": 0, "after": (2, 64, 3, 1)}
        bad = Tuning(1, 0, 0, 64, 0, 7, 0)  # decode_tiling 7 is invalid
        assert L.xec_set_tuning(ctypes.byref(bad)) == xec.Status.INVALID_SIZE
        u = Tuning()
        L.xec_get_tuning(ctypes.byref(u))
        assert (u.unroll, u.max_grid, u.block_threads, u.decode_tiling) == (2, 64, 256, 3)
        assert L.xec_get_tuning(None) == xec.Status.INVALID_ALIGNMENT
        assert L.xec_set_tuning(None) == xec.Status.INVALID_ALIGNMENT
    finally:
        assert L.xec_set_tuning(ctypes.byref(Tuning())) == 0  # back to the defaults


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_header_is_plain_c_and_links(tmp_path):
    """The boundary is a C ABI: include/xec.h compiles as strict C99 (no C++,
    no HIP headers needed: hipStream_t is an opaque pointer), and a C program
    links against libxec_hip.so and runs its host-only entry points -- the
    reference's argument checks (xorec_utils.hpp:61-86) and recoverability scan
    (:144-175) -- without a GPU."""
    src = tmp_path / "c_client.c"
    src.write_text(r'''
#include <stdio.h>
#include <stdlib.h>
#include "xec.h"
int main(void) {
  static unsigned char bm[2 * 5];
  int needs = -1;
  void* data = (void*)(uintptr_t)64;  /* only the address is checked */
  for (int i = 0; i < 10; ++i) bm[i] = 1;
  if (xec_check_args(data, data, 4096, 4, 1) != XEC_SUCCESS) return 1;
  if (xec_check_args(data, data, 100, 4, 1) != XEC_INVALID_SIZE) return 2;
  if (xec_check_args((void*)(uintptr_t)65, data, 4096, 4, 1) != XEC_INVALID_ALIGNMENT) return 3;
  if (xec_check_args(data, data, 4096, 6, 4) != XEC_INVALID_COUNTS) return 4;
  bm[5 + 2] = 0;  /* stripe 1 lost data block 2 */
  if (xec_check_bitmap(bm, 2, 4, 1, &needs) != XEC_SUCCESS || needs != 1) return 5;
  bm[5 + 4] = 0;  /* ... and its class parity: unrecoverable */
  if (xec_check_bitmap(bm, 2, 4, 1, &needs) != XEC_DECODE_FAILURE) return 6;
  printf("%s %s\n", xec_status_string(XEC_DECODE_FAILURE), xec_build_info());
  return 0;
}
''')
    exe = tmp_path / "c_client"
    lib_dir = xec.LIB_PATH.parent
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic",
                    f"-I{ROOT / 'include'}", str(src), "-o", str(exe), f"-L{lib_dir}",
                    "-lxec_hip", f"-Wl,-rpath,{lib_dir}"], check=True, capture_output=True)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, (p.returncode, p.stderr)
    assert p.stdout.startswith("DecodeFailure xec-hip gfx950")


def test_select_lost_blocks_matches_oracle(oracle):
    """xec_select_lost_blocks (host only) == the oracle's restatement of the
    reference's select_lost_blocks (utils.cpp:100-127) with the same seed, and
    every draw is recoverable (at most one loss per parity class)."""
    import numpy as np

    import xorec_oracle as xo
    for k, m in [(4, 1), (16, 1), (8, 4), (32, 8), (16, 16), (5, 5), (64, 2)]:
        for lost in range(0, m + 1):
            for seed in (0, 1, 7, 1896, 2**40 + 3):
                got = np.ones(k + m, np.uint8)
                assert xec.select_lost_blocks(k, m, lost, got, seed) == xec.Status.SUCCESS
                want = np.ones(k + m, np.uint8)
                assert xo.np_select_lost_blocks(k, m, lost, want, seed) == 0
                assert (got == want).all(), (k, m, lost, seed)
                zeros = np.flatnonzero(got == 0)
                assert len(zeros) == lost and len(set(zeros % m)) == lost
    bm = np.ones(5, np.uint8)
    assert xec.select_lost_blocks(4, 1, 2, bm, 0) == xec.Status.INVALID_COUNTS
    assert (bm == 1).all()


def test_pipeline_create_rejects_bad_sizes_before_the_device():
    # argument checks (xorec_utils.hpp:61-86 on bs, k, m) and a slot size
    # chunk_stripes*(k+m)*bs that must fit a size_t come before any HIP call,
    # so they answer without a GPU and leave nothing allocated
    import ctypes
    L = xec.lib()
    h = ctypes.c_void_p(123)
    cases = [
        ((4, 100, 4, 1, 2), xec.Status.INVALID_SIZE),     # bs not a multiple of 256
        ((4, 4096, 6, 4, 2), xec.Status.INVALID_COUNTS),  # k % m != 0
        ((0, 4096, 4, 1, 2), xec.Status.INVALID_SIZE),    # no stripes per chunk
        ((4, 4096, 4, 1, 0), xec.Status.INVALID_SIZE),    # no streams
        ((4, 4096, 4, 1, 17), xec.Status.INVALID_SIZE),   # more than 16 streams
        ((2**62, 4096, 16, 1, 2), xec.Status.INVALID_SIZE),  # slot bytes overflow
        ((1, 2**60, 32, 32, 2), xec.Status.INVALID_SIZE),    # row bytes overflow
    ]
    for args, want in cases:
        h.value = 123
        assert xec.Status(L.xec_pipeline_create(ctypes.byref(h), *args)) == want, args
        assert h.value is None, args  # *out cleared on every failure
