"""The reference-side plugins against the reference's UNMODIFIED plugin interface.

integration/xorec_hip_bm.{hpp,cpp} (one GPU) and xorec_hip_multi_bm.{hpp,cpp}
(the batch over several GPUs of one process, devices from XEC_DEVICES; no new
BenchmarkConfig field, bm_config.hpp:25-43) are the classes a maintainer adds
to the reference's src/algorithms/ (INTEGRATION.md §2, §3).  This test compiles it together
with the reference's own abstract_bm.cpp and utils.cpp, where they lie under
/root/reference (abstract_bm.hpp:18-88, abstract_bm.cpp:4-61, utils.cpp:35-127),
and links it against libxec_hip.so (integration/Makefile; output under a
temporary directory, never in the repository or on the GPU box).  CPU only:
the binary is linked, not run.  Skipped where the reference is not mounted.
"""
from __future__ import annotations

import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference")
LIB = ROOT / "erasure-code-benchmark_amd" / "xec" / "libxec_hip.so"

pytestmark = pytest.mark.skipif(not (REF / "src" / "algorithms" / "abstract_bm.hpp").exists(),
                                reason="reference not mounted (the GPU box never has it)")

OVERRIDES = ["XorecBenchmarkHip::setup()", "XorecBenchmarkHip::encode()",
             "XorecBenchmarkHip::decode()", "XorecBenchmarkHip::simulate_data_loss()",
             "XorecBenchmarkHip::check_for_corruption() const",
             "XorecBenchmarkHip::m_write_data_buffer()"]


@pytest.fixture(scope="module")
def built(tmp_path_factory):
    if not LIB.exists():
        pytest.skip("libxec_hip.so not built")
    out = tmp_path_factory.mktemp("xec_ref_integration")
    r = subprocess.run(["make", "-C", str(ROOT / "integration"), f"OUT={out}"],
                       capture_output=True, text=True)
    if "no cuda_runtime.h in image" in r.stdout + r.stderr:
        pytest.skip("NVIDIA cuda_runtime.h (triton) absent: reference headers unbuildable")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return out


MULTI_OVERRIDES = [o.replace("XorecBenchmarkHip::", "XorecBenchmarkHipMulti::") for o in OVERRIDES]


def _nm(path, *flags):
    return subprocess.run(["nm", "-C", *flags, str(path)], capture_output=True, text=True,
                          check=True).stdout


def test_plugin_overrides_every_virtual(built):
    # `override` on each declaration already makes a signature mismatch with
    # the reference's AbstractBenchmark a compile error; nm shows the bodies exist
    syms = _nm(built / "xorec_hip_bm.o")
    for name in OVERRIDES:
        assert f" T {name}" in syms, name
    assert "vtable for XorecBenchmarkHip" in syms


def test_multi_plugin_overrides_every_virtual(built):
    syms = _nm(built / "xorec_hip_multi_bm.o")
    for name in MULTI_OVERRIDES:
        assert f" T {name}" in syms, name
    assert "vtable for XorecBenchmarkHipMulti" in syms
    # config 5's exchange and the device list (XEC_DEVICES), no config field
    for name in ("XorecBenchmarkHipMulti::scatter_from(unsigned char const*, int)",
                 "XorecBenchmarkHipMulti::gather_parity_to(unsigned char*, int)"):
        assert f" T {name}" in syms, name
    assert "XEC_DEVICES" in (ROOT / "integration" / "xorec_hip_multi_bm.cpp").read_text()


def test_reference_config_is_unmodified():
    """The plugins use the reference's BenchmarkConfig as it is: every field
    they read exists in bm_config.hpp:25-43 (no `devices`, no `seed`)."""
    import re
    fields = set(re.findall(r"^\s+[\w:<>*]+\s+(\w+)(?:\s*=[^;]*)?;",
                            (REF / "src/benchmark/bm_config.hpp").read_text(), re.M))
    for f in ("xorec_hip_bm.cpp", "xorec_hip_multi_bm.cpp", "ref_plugin_main.cpp"):
        used = set(re.findall(r"(?<![\w])config\.(\w+)", (ROOT / "integration" / f).read_text()))
        assert used <= fields, (f, used - fields)


def test_links_reference_interface_with_libxec(built):
    exe = built / "ref_plugin_main"
    assert exe.exists()
    undef = _nm(exe, "-u")
    # the codec calls go to libxec_hip.so's C ABI, nothing to a CUDA runtime
    for fn in ("xec_init", "xec_encode", "xec_decode", "xec_erase", "xec_validate_blocks",
               "xec_check_bitmap"):
        assert f" U {fn}" in undef, fn
    assert "cuda" not in undef.lower()
    # the reference's own interface code is what got linked, not this repo's mirror
    defined = _nm(exe)
    assert "AbstractBenchmark::AbstractBenchmark(BenchmarkConfig const&)" in defined
    assert "select_lost_blocks(unsigned long, unsigned long, unsigned long, unsigned char*)" in defined
    assert "write_validation_pattern(unsigned char*, unsigned long)" in defined
    assert "xec::" not in defined
    ldd = subprocess.run(["ldd", str(exe)], capture_output=True, text=True).stdout
    assert "libxec_hip.so" in ldd and "not found" not in ldd.split("libxec_hip.so")[1].split("\n")[0]


def test_nothing_from_the_reference_travels():
    """Built objects land in the temporary OUT only (integration/Makefile)."""
    assert not list((ROOT / "integration").glob("*.o"))
    assert not (ROOT / "integration" / "ref_plugin_main").exists()
