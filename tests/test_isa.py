"""ISA-level invariants of the gfx950 kernels (CPU only: hipcc cross-compiles).

* every load of a non-temporal (NT=true) encode/decode instantiation carries
  `nt` and every result store its kernel's policy (encode `nt`, decode `sc1`)
  -- hipcc has been seen to drop `nt` silently (xec_kernels.hip, st16_block),
  which cost 5 % of bandwidth;
* the benchmark-shape kernels' registers admit the residency the launch asks
  for by default (auto_occupancy in csrc/xec_api.cpp), and the 32-member
  kernels issue all their loads before the first wait.
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
    for m in re.finditer(r"^(_ZN3xec[12][0-9](encode|decode)_(?:class_|list_|arglist_|argmask_|devlist_)?kernel\w+):.*?^\s*s_endpgm", text,
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


def test_nt_kernels_carry_their_cache_policy(kernels):
    """Every load of an NT kernel is `nt`; its result stores carry the policy
    chosen per kernel (xec_kernels.hip kEncodeStoreAux / kDecodeStoreAux):
    encode `nt`, decode `sc1` (not kept in L2)."""
    for name, k in kernels.items():
        if not _nt(name):
            continue
        loads = re.findall(r"^\s*((?:global|buffer)_load_dwordx4[^\n]*)", k["body"], re.M)
        stores = re.findall(r"^\s*((?:global|buffer)_store_dwordx4[^\n]*)", k["body"], re.M)
        assert loads and stores, name
        missing = [i for i in loads if not re.search(r"\bnt\b", i)]
        assert not missing, f"{name}: {missing[:3]}"
        want = r"\bsc1\b" if "decode_" in name else r"\bnt\b"
        wrong = [i for i in stores if not re.search(want, i)]
        assert not wrong, f"{name}: {wrong[:3]}"
        if "decode_" in name:
            assert not [i for i in stores if re.search(r"\bnt\b", i)], name


# member count -> resident waves per SIMD the launch asks for by default
# (auto_occupancy, csrc/xec_api.cpp); the kernel's registers must admit them.
AUTO_OCCUPANCY = {4: 4, 8: 4, 16: 2, 32: 1}


@pytest.mark.parametrize("kind", ["encode", "decode", "decode_class", "decode_list",
                                  "decode_arglist", "decode_argmask", "decode_devlist"])
@pytest.mark.parametrize("nm", sorted(AUTO_OCCUPANCY))
def test_registers_admit_the_default_residency(kernels, kind, nm):
    hits = [k for n, k in kernels.items()
            if re.search(rf"{kind}_kernelILi{nm}ELi1ELb1ELi64E", n)]
    assert hits
    for k in hits:
        vgpr_alloc = -(-k["vgpr"] // 8) * 8  # gfx950 allocates VGPRs in blocks of 8
        assert 512 // vgpr_alloc >= AUTO_OCCUPANCY[nm], k["vgpr"]
        assert k["sgpr"] <= 96, k["sgpr"]


def test_32_member_kernels_issue_every_load_before_the_first_wait(kernels):
    """NM=32 keeps all class loads in flight (sched_barrier after the load
    loop): 32 global loads precede the first vmcnt wait of the unrolled path."""
    for name, k in kernels.items():
        if not re.search(r"(en|de)code_kernelILi32ELi1ELb1ELi64E", name):
            continue
        body = k["body"]
        first_load = body.index("global_load_dwordx4")
        first_wait = body.index("s_waitcnt vmcnt", first_load)
        assert body[first_load:first_wait].count("global_load_dwordx4") == 32, name
