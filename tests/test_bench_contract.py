"""bench.py keeps the driver's contract: one JSON line with the required keys,
roofline + cpu_baseline objects, verified results (GPU, small sizes)."""
from __future__ import annotations

import json
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
            "roofline", "cpu_baseline"}


def run_bench(*args):
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True,
                       text=True, timeout=600, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    # stdout carries exactly the result line (RCCL's init banner and any other
    # library output go to stderr: bench.py _result_stream)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("workload,stripes", [("cfg3", 16), ("cfg2", 64), ("cfg4", 512)])
def test_bench_json_line(workload, stripes):
    out = run_bench("--workload", workload, "--stripes", str(stripes), "--steps", "3",
                    "--warmup", "1", "--cpu-seconds", "0.5")
    assert REQUIRED <= set(out)
    assert out["verified"] is True
    assert out["n_gpus"] == 1 and out["steps"] == 3 and out["warmup"] == 1
    assert out["unit"] == "GB/s" and out["higher_is_better"] is True
    assert out["scaling"] == "weak" and out["dtype"] == "u8"
    assert out["config"]["workload"].startswith(workload)
    r = out["roofline"]
    assert r["bound"] == "hbm" and r["peak"] == 8000.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    c = out["cpu_baseline"]
    assert c["kind"] == "port" and c["cores"] >= 1 and c["value"] > 0
    assert c["single_thread"]["value"] > 0
    assert set(c["by_workload"]) == {"cfg2", "cfg3", "cfg4"}
    # value = the fastest measured placement; by_workload is the GPU-node-bound child's
    assert c["by_workload"][workload]["value"] == c["gpu_node_bound_diagnostic"]["value"]
    assert c["value"] == max(c["placements"].values())
    assert out["value"] > 0
    assert abs(out["value_frac_of_n_gpu_hbm_peak"] - out["value"] / 8000.0) < 1e-3
    by_set = out["median_ms_by_set_rank0"]  # placement is visible per resident set
    assert all(len(by_set[n]) == 3 and all(t > 0 for t in by_set[n]) for n in ("encode", "decode"))
    assert out["dist"]["ranks_seen"] == 1 and len(out["per_rank"]) == 1
    hp = out["host_pipeline"]  # the north star's host-in / host-out leg
    assert hp["bit_exact"] is True and "error" not in hp, hp
    assert hp["encode_GBps_data"] > 0 and hp["decode_GBps_data"] > 0
    assert len(hp["per_rank_numa_node"]) == 1  # -1 where sysfs names no node
    pg = hp["pageable"]  # the same batch from pageable buffers (file / socket buffers)
    assert pg["bit_exact"] is True and pg["encode_GBps_data"] > 0 and pg["decode_GBps_data"] > 0


def test_bench_device_decode_api():
    out = run_bench("--workload", "cfg2", "--stripes", "64", "--steps", "3", "--warmup", "1",
                    "--no-cpu-baseline", "--decode-api", "device")
    assert out["verified"] is True and out["value"] > 0
    assert out["config"]["decode_api"] == "xec_decode_device"
    stats = out["launch_stats_rank0"]
    assert set(stats) == {"encode", "decode"}
    assert stats["decode"]["min_ms"] <= stats["decode"]["median_ms"] <= stats["decode"]["max_ms"]


def test_bench_multi_erasure_line():
    """--lost 4 at k=16+4: four data blocks lost per stripe (one per class),
    decode bytes scale with the erasures, verification still bit-exact."""
    out = run_bench("--workload", "16,4,65536,64", "--lost", "4", "--steps", "3", "--warmup", "1",
                    "--no-cpu-baseline")
    assert out["verified"] is True and out["value"] > 0
    assert out["config"]["erasure"].startswith("4 data blocks lost")
    assert out["roofline_by_kernel"]["decode"]["algorithmic_bytes_per_launch"] == 4 * 64 * 5 * 65536


def test_bench_graph_leg():
    """--graph replays one captured rotation of encode + device decode steps;
    the headline line is unchanged and verification still passes."""
    out = run_bench("--workload", "cfg2", "--stripes", "64", "--steps", "6", "--warmup", "1",
                    "--no-cpu-baseline", "--decode-api", "device", "--graph")
    assert out["verified"] is True and out["value"] > 0
    g = out["graph"]
    assert g["steps"] == 6 and g["ms_per_step"] > 0


def test_bench_rccl_world1():
    """The RCCL code path on the one-GPU box: a one-rank nccl process group,
    barrier / all_gather around the timed region and the scatter/gather leg."""
    out = run_bench("--workload", "cfg2", "--stripes", "64", "--steps", "3", "--warmup", "1",
                    "--no-cpu-baseline", "--dist-world1")
    assert out["verified"] is True
    assert out["dist"]["backend"] == "nccl" and out["dist"]["ranks_seen"] == 1
    sc = out["scatter"]
    assert sc.get("bit_exact") is True, sc
    assert sc["gathered_parity_bit_exact_vs_root_encode"] is True
    # the topology record at world 1: the root reaches only itself
    assert out["topology"]["path"] == "local" and sc["path"] == "local", out["topology"]
    assert out["host_pipeline"]["bit_exact"] is True


def test_bench_launcher_two_ranks_one_gpu():
    """`bench.py --gpus 2` starts both ranks itself; on one GPU they share the
    device under gloo (RCCL refuses two ranks per device)."""
    out = run_bench("--gpus", "2", "--dist-backend", "gloo", "--workload", "cfg2", "--stripes",
                    "32", "--steps", "3", "--warmup", "1")
    assert out["n_gpus"] == 2 and out["verified"] is True
    assert out["dist"] == {"backend": "gloo", "ranks_seen": 2, "launcher": "bench.py"}
    assert out["config"]["stripes_total"] == 64 and len(out["per_rank"]) == 2
    hp = out["host_pipeline"]  # both ranks stream their own host batch at once
    assert hp["bit_exact"] is True and len(hp["per_rank_encode_GBps_data"]) == 2, hp


def test_bench_default_roofline_recomputes_from_profile():
    """At the default workload the line's roofline.frac is this run's HIP-event
    figure (the contract), and its rocprof_profile.frac is algorithmic bytes /
    the rocprofv3 AverageNs of the kernel-stats CSV it cites (profiles/), to 3
    decimals; the two clocks agree within the device spread."""
    import csv
    out = run_bench("--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-host-pipeline")
    r = out["roofline"]
    assert r["timing_source"].startswith("HIP events"), r
    assert 0 < r["frac"] < 1 and r["avg_launch_ms"] > 0
    rp = r["rocprof_profile"]
    path = ROOT / rp["source"].rsplit(": ", 1)[1]
    base = r["kernel"].split("<")[0]
    row = [x for x in csv.DictReader(open(path))
           if x["Name"].split("(")[0].replace("void ", "").split("<")[0] == base][0]
    frac = r["algorithmic_bytes_per_launch"] / float(row["AverageNs"]) / 8000.0
    assert round(frac, 3) == round(rp["frac"], 3)
    assert 0.85 < rp["over_hip_events_ms"] < 1.15, r
