"""Host code under AddressSanitizer + UBSan (CPU only; GPU sanitizers are not
available on this pool): the batch recoverability scan of xec_decode, fuzzed
against a direct restatement of the reference rules with exact-size buffers
(an over-read of the caller's bitmap fails the test), and the oracle's C
restatement."""
from __future__ import annotations

import shutil
import subprocess

import pytest

from conftest import ROOT, run_tsan


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_scan_fuzz_asan_ubsan(tmp_path):
    exe = tmp_path / "scan_fuzz"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", f"-I{ROOT / 'include'}",
                    str(ROOT / "tests" / "host" / "scan_fuzz.cpp"),
                    str(ROOT / "erasure-code-benchmark_amd" / "csrc" / "xec_scan.cpp"),
                    "-o", str(exe)], check=True, capture_output=True)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "scan_fuzz ok" in p.stdout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_asan_ubsan(tmp_path):
    """The oracle itself (the parity checker) under ASan/UBSan: known answers
    and erase/decode round trips with exact-size buffers."""
    exe = tmp_path / "oracle_asan"
    subprocess.run(["gcc", "-std=c11", "-O1", "-g", "-fopenmp", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", f"-I{ROOT / 'oracle'}",
                    str(ROOT / "tests" / "host" / "oracle_asan.c"),
                    str(ROOT / "oracle" / "xorec_oracle.c"), "-o", str(exe)],
                   check=True, capture_output=True)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "oracle_asan ok" in p.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_shard_pool_tsan(tmp_path):
    """The multi-device plugin's per-shard decode threads (integration/shard_pool.hpp)
    under ThreadSanitizer: each run calls every shard once and returns after
    all of them, over 2,000 runs per pool size."""
    exe = tmp_path / "shard_pool_test"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread",
                    f"-I{ROOT / 'integration'}",
                    str(ROOT / "tests" / "host" / "shard_pool_test.cpp"), "-o", str(exe)],
                   check=True, capture_output=True)
    p = run_tsan([str(exe)], timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "shard_pool ok" in p.stdout
