"""bench.py's roofline object.

`roofline.achieved` / `frac` = algorithmic bytes per launch / the kernel's
average launch duration measured live with HIP events in the run itself;
beside it, `rocprof_profile` = the same from the rocprofv3 AverageNs in the
kernel-stats CSV that profiles/traffic_<workload>.json names as its
`timing_source` (the same profiling session as its PMC bytes), recomputable
from profiles/ alone.  CPU only: bench.roofline is called with a made-up
HIP-event time, and the expected figures are recomputed here straight from the
cited CSV.
"""
from __future__ import annotations

import csv
import json

import pytest

from conftest import ROOT

import bench


def _row(path, base):
    for r in csv.DictReader(open(ROOT / path)):
        if r["Name"].split("(")[0].replace("void ", "").split("<")[0] == base:
            return r
    raise AssertionError(f"{base} not in {path}")


@pytest.mark.parametrize("workload", sorted(bench.WORKLOADS))
def test_frac_recomputes_from_cited_profile(workload):
    k, m, bs, S, _ = bench.WORKLOADS[workload]
    b_enc, b_dec = bench.algorithmic_bytes(S, k, m, bs)
    _, src = bench.load_traffic(workload)
    assert src is not None and src["encode_algorithmic_bytes_per_launch"] == b_enc
    assert (ROOT / src["timing_source"]).exists()
    # the timing source and the traffic source are one profiling session (one tag)
    assert src["timing_source"].replace("_kernel_stats.csv", "") in src["source"]
    dec_base = src["decode_kernel"].split("<")[0]
    for base, b, hbm in (("xec::encode_kernel", b_enc, src["encode_hbm_bytes_per_launch"]),
                         (dec_base, b_dec, src["decode_hbm_bytes_per_launch"])):
        r = bench.roofline(base, b, 1.0, hbm, src)
        # the headline: this run's HIP events (here a made-up 1 ms)
        assert r["avg_launch_ms"] == 1.0 and r["timing_source"].startswith("HIP events")
        assert abs(r["frac"] - b / 1e-3 / 1e9 / 8000.0) < 1e-4
        # beside it, the committed profile's rocprofv3 average, to 4 places
        rp = r["rocprof_profile"]
        avg_ns = float(_row(src["timing_source"], base)["AverageNs"])
        assert abs(b / avg_ns / 8000.0 - rp["frac"]) < 1e-4
        assert rp["avg_launch_ms"] == round(avg_ns * 1e-6, 4)
        assert src["timing_source"] in rp["source"]
        assert rp["over_hip_events_ms"] == round(avg_ns * 1e-6 / 1.0, 4)
        assert r["traffic"] == hbm and r["traffic_source"] == src["source"]


def test_frac_without_a_profile():
    r = bench.roofline("xec::encode_kernel", 8_000_000_000, 1.0, None, None)
    assert r["timing_source"].startswith("HIP events")
    assert r["frac"] == 1.0 and "rocprof_profile" not in r
    # a profile that lacks the kernel (e.g. a forced decode tiling) has no cross-check
    src = json.loads((ROOT / "profiles" / "traffic_cfg3.json").read_text())
    r = bench.roofline("xec::decode_class_kernel", 8_000_000_000, 1.0, None, src)
    assert r["frac"] == 1.0 and "rocprof_profile" not in r


def _source_id():
    """erasure-code-benchmark_amd/Makefile's XEC_SRC_ID: sha256 of the library's
    sources (sorted csrc/*.hip, *.cpp, *.h), include/xec.h, the Makefile, the
    compiler flags and `hipcc --version`, as make computes it."""
    import subprocess
    out = subprocess.run(["make", "-s", "-C", str(ROOT / "erasure-code-benchmark_amd"),
                          "print-id"], capture_output=True, text=True, check=True).stdout
    return out.strip().splitlines()[-1]


def test_library_build_id_is_its_sources():
    """xec_build_info()'s "src:<id>" is the hash of the sources, flags and
    compiler in the tree, so the id names what the library was built from (no
    stale .so)."""
    import xec
    sid = _source_id()
    assert len(sid) == 16 and int(sid, 16) >= 0
    assert bench.build_id_of(xec.build_info()) == sid


@pytest.mark.parametrize("workload", sorted(bench.WORKLOADS))
def test_profile_is_the_shipped_library(workload):
    """the profile behind the line's frac recorded the
    build id of the library that ships; bench.py reports the comparison."""
    import xec
    lib = bench.build_id_of(xec.build_info())
    _, src = bench.load_traffic(workload)
    assert lib and src.get("build_id") == lib, (src.get("build_id"), lib)
    pmc = json.loads((ROOT / src["source"].split(" ")[0]).read_text())
    assert pmc["build_id"] == lib
    assert (ROOT / src["timing_source"]).exists()
    r = bench.roofline("xec::encode_kernel", 1, 1.0, None, src, lib)
    assert r["profile_is_this_library"] is True and r["profile_build_id"] == lib
