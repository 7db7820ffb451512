"""`python bench.py --gpus N` starts its own ranks.

Run as a plain command, the way the driver runs `--gpus 1`, with the explicit
CPU rehearsal (`--rehearse-cpu --dist-backend gloo`: tools/cpu_rehearsal.py
stands in for every device call).  What is checked is the launcher and the N>1
bookkeeping -- rank environment, rendezvous on 127.0.0.1, one JSON line from
rank 0 only, max-over-ranks timing, per-rank rates, the scatter/gather leg and
exit-status propagation -- not any number.
"""
from __future__ import annotations

import json
import subprocess
import sys

import pytest

from conftest import ROOT


def _bench(*args, timeout=300):
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True,
                          text=True, timeout=timeout, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 4, 8])  # 8: the driver's largest scaling run
def test_launcher_plain_command(n):
    p = _bench("--gpus", str(n), "--rehearse-cpu", "--dist-backend", "gloo",
               "--workload", "8,2,4096,5", "--steps", "3", "--warmup", "1")
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout  # rank 0's line, nothing else
    out = json.loads(lines[0])
    assert out["n_gpus"] == n
    assert out["dist"] == {"backend": "gloo", "ranks_seen": n, "launcher": "bench.py"}
    assert out["config"]["stripes_total"] == 5 * n
    assert [r["rank"] for r in out["per_rank"]] == list(range(n))
    assert all(r["stripes"] == 5 for r in out["per_rank"])
    assert [r["device"] for r in out["per_rank"]] == [0] * n  # CPU stand-ins: one "device"
    assert out["verified"] is True
    assert out["data"].startswith("CPU REHEARSAL")
    assert out["cpu_baseline"] is None  # the CPU leg is N=1 only
    # the whole-job rate against the N GPUs' HBM together (north star)
    assert abs(out["value_frac_of_n_gpu_hbm_peak"] - out["value"] / (n * 8000.0)) < 1e-3
    sc = out["scatter"]
    assert sc["bit_exact"] is True and sc["gathered_parity_bit_exact_vs_root_encode"] is True
    # max-over-ranks: the reported step time covers every rank's elapsed time
    assert out["ms_per_step"] * out["steps"] >= max(r["elapsed_ms"] for r in out["per_rank"]) - 1e-3
    # the one-process multi-device leg: a child started by
    # rank 0 after every rank finished, over the N devices the ranks ran on
    md = out["multi_device"]
    assert md["rehearsal"] is True and md["devices"] == [0] * n  # CPU stand-ins: one "device"
    assert md["stripes_per_device"] == 5 and md["stripes_total"] == 5 * n
    assert md["bit_exact"] is True
    assert md["scatter"]["gathered_parity_bit_exact_vs_root_encode"] is True
    assert "error" not in md


def test_torchrun_launch_one_line():
    """Launched the way the driver launches N > 1 (torch.distributed.run, one rank
    per process, WORLD_SIZE set): still exactly one line on stdout."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "4", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), str(ROOT / "bench.py"), "--gpus", "4", "--rehearse-cpu",
                        "--dist-backend", "gloo", "--workload", "8,2,4096,5", "--steps", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 4 and out["dist"]["ranks_seen"] == 4
    assert out["dist"]["launcher"] == "external"
    # under an external launcher rank 0 starts the multi-device leg itself
    assert out["multi_device"]["bit_exact"] is True and out["multi_device"]["devices"] == [0] * 4


def test_multi_device_leg_at_n1_with_a_device_list():
    """--multi-devices 0,0 runs the leg at N=1 (how a one-GPU box rehearses
    config 5's plugin with a repeated device list); still one stdout line."""
    p = _bench("--rehearse-cpu", "--dist-backend", "gloo", "--workload", "4,1,4096,3",
               "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--multi-devices", "0,0")
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout
    md = json.loads(lines[0])["multi_device"]
    assert md["devices"] == [0, 0] and md["bit_exact"] is True and md["stripes_total"] == 6


def test_multi_device_leg_timeout_costs_the_field_not_the_line():
    p = _bench("--gpus", "2", "--rehearse-cpu", "--dist-backend", "gloo", "--workload",
               "8,2,4096,5", "--steps", "2", "--warmup", "1", "--multi-timeout", "0.01")
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert "timed out" in out["multi_device"]["error"]
    assert out["verified"] is True and out["value"] > 0


def test_multi_device_leg_off():
    p = _bench("--gpus", "2", "--rehearse-cpu", "--dist-backend", "gloo", "--workload",
               "8,2,4096,5", "--steps", "2", "--warmup", "1", "--multi-devices", "none")
    assert p.returncode == 0, p.stderr[-3000:]
    assert "multi_device" not in json.loads(p.stdout.strip())


def test_launcher_propagates_rank_failure():
    # every rank refuses (--rehearse-cpu needs gloo): the launcher must fail too
    p = _bench("--gpus", "2", "--rehearse-cpu", "--dist-backend", "nccl", "--steps", "1",
               "--warmup", "0", "--rank-grace", "5", timeout=120)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("gpus", [1, 2])
def test_hung_leg_is_visible_in_exit_status(gpus):
    """The legs' watchdog (--scatter-timeout) fires while the scatter leg runs
    (held up for longer than the watchdog by --rehearse-leg-delay; a bare short
    watchdog raced a tiny leg that could finish first):
    rank 0 still prints exactly one line, carrying the leg's error, and the
    command -- the bench.py launcher at N=2, the lone rank at N=1 -- exits 3."""
    extra = ["--dist-world1"] if gpus == 1 else []
    p = _bench("--gpus", str(gpus), *extra, "--rehearse-cpu", "--dist-backend", "gloo",
               "--workload", "8,2,4096,5", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
               "--scatter-timeout", "0.5", "--rehearse-leg-delay", "30", timeout=180)
    assert p.returncode == 3, (p.returncode, p.stderr[-3000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout
    out = json.loads(lines[0])
    assert "timed out" in out["scatter"]["error"]
    assert out["verified"] is True and out["value"] > 0


def test_world1_process_group_rehearsal():
    """--dist-world1 opens a one-rank group and runs the collectives + scatter leg."""
    p = _bench("--rehearse-cpu", "--dist-backend", "gloo", "--dist-world1",
               "--workload", "4,1,4096,3", "--steps", "2", "--warmup", "1", "--no-cpu-baseline")
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 1 and out["dist"]["ranks_seen"] == 1
    assert out["scatter"]["bit_exact"] is True


@pytest.mark.parametrize("stub,path", [("xgmi", "xgmi-p2p"), ("staged", "staged")])
def test_topology_record_in_the_line(stub, path):
    """the N > 1 line records, per root -> peer pair, peer
    access, link type and hops, and labels the scatter "xgmi-p2p" or "staged"
    from that record -- here from a stubbed topology (XEC_TOPOLOGY_STUB), since
    the CPU has no runtime to ask."""
    import os
    env = dict(os.environ, XEC_TOPOLOGY_STUB=stub)
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4", "--rehearse-cpu",
                        "--dist-backend", "gloo", "--workload", "8,2,4096,5", "--steps", "2",
                        "--warmup", "1", "--multi-devices", "none"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    topo = out["topology"]
    assert topo["root"] == 0 and [q["device"] for q in topo["pairs"]] == [0, 1, 2, 3]
    assert topo["pairs"][0]["path"] == "local"
    assert all(q["path"] == path for q in topo["pairs"][1:])
    assert topo["path"] == path and "STUB" in topo["source"]
    assert out["scatter"]["path"] == path


def test_topology_record_needs_a_runtime_or_a_stub():
    import os
    env = {k: v for k, v in os.environ.items() if k != "XEC_TOPOLOGY_STUB"}
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--rehearse-cpu",
                        "--dist-backend", "gloo", "--workload", "8,2,4096,5", "--steps", "2",
                        "--warmup", "1", "--multi-devices", "none"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert "skipped" in out["topology"] and out["scatter"]["path"] == "unknown"


@pytest.mark.parametrize("stub,path", [("xgmi", "xgmi-p2p"), ("staged", "staged")])
def test_multi_leg_stand_in_topology(stub, path):
    """The multi_device leg's record (host/xec_multi_leg.cpp: "topology" and the
    scatter's "path"), from the CPU stand-in over a stubbed 4-GPU node."""
    import os
    env = dict(os.environ, XEC_TOPOLOGY_STUB=stub)
    p = subprocess.run([sys.executable, str(ROOT / "tools" / "cpu_rehearsal.py"), "multi-leg",
                        "--devices", "0,1,2,3", "--stripes-per-device", "2", "--data", "4",
                        "--block", "4096"], capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["topology"]["path"] == path and out["scatter"]["path"] == path
    assert [q["path"] for q in out["topology"]["pairs"]] == ["local"] + [path] * 3
