"""The plugin interface's default behaviour (integration/iface/abstract_bm.{hpp,cpp},
restating the reference's abstract_bm.hpp:18-88 and abstract_bm.cpp:4-60):
a CPU plugin that overrides only setup / encode / decode runs clean through
the harness loop, and the default corruption check catches a skipped decode.
CPU only (g++), also under ASan/UBSan."""
from __future__ import annotations

import shutil
import subprocess

import pytest

from conftest import ROOT

HOST = ROOT / "erasure-code-benchmark_amd" / "host"
IFACE = ROOT / "integration" / "iface"


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("sanitize", [False, True])
def test_plugin_defaults(tmp_path, sanitize):
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"] if sanitize else []
    obj = tmp_path / "oracle.o"
    subprocess.run(["gcc", "-std=c11", "-O1", "-g", "-fopenmp", *san, "-c",
                    str(ROOT / "oracle" / "xorec_oracle.c"), "-o", str(obj)], check=True)
    exe = tmp_path / "plugin_defaults"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fopenmp", *san, f"-I{HOST}",
                    f"-I{IFACE}", f"-I{ROOT / 'integration'}", f"-I{ROOT / 'oracle'}",
                    str(ROOT / "tests" / "host" / "plugin_defaults.cpp"),
                    str(IFACE / "abstract_bm.cpp"), str(IFACE / "utils.cpp"),
                    str(IFACE / "bm_config.cpp"), str(obj), "-o", str(exe)], check=True)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "plugin_defaults ok" in p.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_restated_interface_utilities_match_the_oracle(tmp_path):
    """integration/iface/utils.cpp (the utilities the plugins' one-argument
    constructor uses) against the oracle: PCG32, the validation payload and
    checksum, the erasure draw (tests/host/iface_utils.cpp)."""
    obj = tmp_path / "oracle.o"
    subprocess.run(["gcc", "-std=c11", "-O1", "-fopenmp", "-c", str(ROOT / "oracle" / "xorec_oracle.c"),
                    "-o", str(obj)], check=True)
    exe = tmp_path / "iface_utils"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fopenmp", "-Wall", "-Wextra", "-Werror",
                    f"-I{IFACE}", f"-I{ROOT / 'oracle'}",
                    str(ROOT / "tests" / "host" / "iface_utils.cpp"), str(IFACE / "utils.cpp"),
                    str(obj), "-o", str(exe)], check=True)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "iface_utils ok" in p.stdout, p.stdout[-3000:] + p.stderr[-3000:]
