"""What travels to the GPU box ("The oracle never travels").

gpurun ships the repository minus the patterns in .gpurunignore.  Anything built
from /root/reference (oracle/_ref, by `make -C oracle ref`) must be among them;
the product libraries, their sources and what the GPU tests load must not be.
"""
from __future__ import annotations

import fnmatch
import re
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _patterns():
    return [ln.strip() for ln in (ROOT / ".gpurunignore").read_text().splitlines()
            if ln.strip() and not ln.startswith("#")]


def _ignored(rel: str) -> bool:
    """tar --exclude semantics as gpurun applies them: './x' anchors at the top
    (and covers everything below x), a bare pattern matches at any depth."""
    for pat in _patterns():
        if pat.startswith("./"):
            p = pat[2:]
            if rel == p or rel.startswith(p + "/") or fnmatch.fnmatch(rel, p):
                return True
        else:
            parts = rel.split("/")
            if any(fnmatch.fnmatch(x, pat) for x in parts) or fnmatch.fnmatch(rel, pat):
                return True
    return False


def test_reference_build_outputs_are_ignored():
    # every file the reference recipe would write, from make's own dry run
    # (without the reference mounted, make cannot plan the rule: read its targets)
    r = subprocess.run(["make", "-n", "-B", "-C", str(ROOT / "oracle"), "ref"],
                       capture_output=True, text=True)
    text = r.stdout if r.returncode == 0 else (ROOT / "oracle" / "Makefile").read_text()
    outs = set(re.findall(r"-o (\$@|\S+)", text)) | set(re.findall(r"mkdir -p (\S+)", text))
    outs |= set(re.findall(r"^(_ref/\S+):", text, re.M))
    outs.discard("$@")
    assert outs, r.stdout + r.stderr
    for o in outs:
        rel = str((ROOT / "oracle" / o).resolve().relative_to(ROOT))
        assert _ignored(rel), f"{rel} (written by make -C oracle ref) would ship to the GPU box"
    assert _ignored("oracle/_ref/ref_driver")


def test_product_and_checkers_travel():
    for rel in ("erasure-code-benchmark_amd/xec/libxec_hip.so",
                "erasure-code-benchmark_amd/xec/libxec_plugin.so",
                "erasure-code-benchmark_amd/csrc/xec_kernels.hip",
                "oracle/liboracle.so", "oracle/xorec_oracle.c", "oracle/xorec_oracle.py",
                "tests/golden/known_answers.json", "bench.py", "__graft_entry__.py",
                "integration/xorec_hip_bm.cpp"):
        assert not _ignored(rel), rel
