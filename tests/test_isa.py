"""ISA-level invariants of the gfx950 kernels (CPU only: hipcc cross-compiles).

* every load and store of a non-temporal (NT=true) encode/decode instantiation
  carries the `nt` cache policy -- hipcc has been seen to drop it silently
  (xec_kernels.hip, st16_block), which cost 5 % of bandwidth;
* the benchmark-shape kernels stay within the register budgets that keep
  8 waves per SIMD resident (MI355X_MICROARCH.md: <= 64 VGPRs, <= 80 SGPRs).
"""
from __future__ import annotations

import re
import subprocess

import pytest

from conftest import PKG_DIR

ASM = PKG_DIR / "build" / "xec_kernels-gfx950.s"


@pytest.fixture(scope="module")
def kernels() -> dict[str, dict]:
    subprocess.run(["make", "-C", str(PKG_DIR), "asm"], check=True, capture_output=True)
    text = ASM.read_text()
    out = {}
    for m in re.finditer(r"^(_ZN3xec1[0-9](encode|decode)_kernel\w+):.*?^\s*s_endpgm", text,
                         re.S | re.M):
        out[m.group(1)] = {"body": m.group(0)}
    meta = re.findall(r"\.name:\s+(\S+)\n(.*?)\.vgpr_count:\s+(\d+)", text, re.S)
    for name, block, vgpr in meta:
        if name in out:
            out[name]["vgpr"] = int(vgpr)
            out[name]["sgpr"] = int(re.search(r"\.sgpr_count:\s+(\d+)", block).group(1))
    assert len(out) >= 100, "kernel instantiations not found in the ISA"
    return out


def _nt(name: str) -> bool:
    # template args <NM, U, NT, T>: ...ILi16ELi1ELb1ELi64E...
    return re.search(r"ELb1E", name) is not None


def test_nt_kernels_use_nt_everywhere(kernels):
    for name, k in kernels.items():
        if not _nt(name):
            continue
        mem = re.findall(r"^\s*((?:global|buffer)_(?:load|store)_dwordx4[^\n]*)", k["body"], re.M)
        assert mem, name
        missing = [i for i in mem if not re.search(r"\bnt\b", i)]
        assert not missing, f"{name}: {missing[:3]}"


@pytest.mark.parametrize("pattern", [r"encode_kernelILi16ELi1ELb1ELi64E",
                                     r"decode_kernelILi16ELi1ELb1ELi64E",
                                     r"encode_kernelILi8ELi1ELb1ELi64E"])
def test_benchmark_shapes_keep_full_occupancy(kernels, pattern):
    hits = [k for n, k in kernels.items() if re.search(pattern, n)]
    assert hits, pattern
    for k in hits:
        assert k["sgpr"] <= 80, k["sgpr"]
        assert k["vgpr"] <= 128, k["vgpr"]
