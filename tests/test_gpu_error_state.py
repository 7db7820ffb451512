"""The caller's pending HIP error across library calls (VERDICT r04 item 3,
ADVICE r04): the library never swallows an error it did not raise, never takes
a failed launch of its own for success, and a query it makes never leaves a
stray NotReady behind.  tests/host/error_preserve.cpp; what the runtime does
with the thread's error state is in tools/lab/last_error_probe.hip
(profiles/r05b/last_error.txt).  The reference checks no CUDA error at all
(/root/reference/src/xorec/xorec_gpu_cmp.cu:45,85-113)."""
from __future__ import annotations

import os
import subprocess

import pytest

from conftest import ROOT

EXE = ROOT / "tests" / "host" / "bin" / "error_preserve"


def _run(mode, **env):
    assert EXE.exists(), "build with make -C tests/host"
    e = dict(os.environ, **env)
    e.pop("XEC_SCRATCH_UPLOADS", None)  # the side-upload path is the one under test
    return subprocess.run([str(EXE), mode], capture_output=True, text=True, timeout=120, env=e)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["decode", "pipeline"])
def test_caller_error_survives_library_calls(mode):
    p = _run(mode)
    assert p.returncode == 0 and f"error_preserve {mode} ok" in p.stdout, p.stdout + p.stderr


@pytest.mark.gpu
def test_failed_launch_is_reported_under_a_same_code_caller_error():
    p = _run("inject", XEC_TEST_FAIL_LAUNCH="1")
    assert p.returncode == 0 and "error_preserve inject ok" in p.stdout, p.stdout + p.stderr
