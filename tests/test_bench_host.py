"""bench.py's host-side pieces on CPU: the algorithmic byte counts behind
`value` / `roofline.achieved` and the CPU-baseline leg's
shape (reference binary when oracle/_ref was built, else the port)."""
from __future__ import annotations

import pytest

import bench


def test_algorithmic_bytes():
    # encode reads k, writes m blocks per stripe; single-erasure decode reads
    # k/m - 1 survivors + 1 parity and writes 1 block
    assert bench.algorithmic_bytes(256, 16, 1, 1 << 20) == (256 * 17 << 20, 256 * 17 << 20)
    assert bench.algorithmic_bytes(4096, 16, 4, 65536) == (4096 * 20 * 65536, 4096 * 5 * 65536)
    assert bench.algorithmic_bytes(1, 4, 1, 4096) == (5 * 4096, 5 * 4096)


def test_workloads_match_baseline_configs():
    k, m, bs, S, desc = bench.WORKLOADS["cfg3"]
    assert (k, m, bs) == (16, 1, 1 << 20) and "configs[2]" in desc
    assert bench.WORKLOADS["cfg2"][:4] == (8, 1, 1 << 16, 1024)
    assert bench.WORKLOADS["cfg4"][:4] == (32, 1, 4096, 65536)


def test_cpu_baseline_shape():
    """The restatement ("port"), never the reference binary; the bench's own
    workload plus the other BASELINE shapes; 1-thread figure beside; median of
    CPU_SAMPLES samples with min / max; threads bound one per core (VERDICT r3
    item 5) and the same threads unbound as a diagnostic."""
    import os
    out = bench.cpu_baseline("cfg2", 8, 1, 1 << 16, 1024, 0.3, 0, sample_bytes=16 << 20)
    assert out["kind"] == "port"
    assert out["unit"] == "GB/s" and out["value"] > 0 and out["cores"] >= 1
    assert out["single_thread"]["value"] > 0
    assert "32 stripes" in out["sample"]  # 16 MiB of k=8 x 64 KiB stripes
    assert len(out["samples"]) == bench.CPU_SAMPLES
    assert out["min"] <= out["value"] <= out["max"]
    assert set(out["by_workload"]) == {"cfg2", "cfg3", "cfg4"}
    # value = the fastest measured placement of the same threads;
    # by_workload comes from the GPU-node-bound child
    assert out["by_workload"]["cfg2"]["value"] == out["gpu_node_bound_diagnostic"]["value"]
    assert out["placement"] in out["placements"]
    assert out["value"] == max(out["placements"].values())
    assert out["placements"]["gpu_node_bound"] == out["gpu_node_bound_diagnostic"]["value"]
    for w in out["by_workload"].values():
        assert w["value"] > 0 and w["single_thread"]["value"] > 0 and w["min"] <= w["max"]
    nproc = len(os.sched_getaffinity(0))
    assert out["nproc"] == nproc and out["cores"] <= nproc
    b = out["binding"]
    assert b["OMP_PROC_BIND"] == "close" and len(b["cpus"]) == out["cores"]
    assert b["OMP_PLACES"] == ",".join("{%d}" % c for c in b["cpus"])
    assert out["unbound_diagnostic"]["value"] > 0
    assert out["by_threads"][str(out["cores"])] == out["value"]
    assert "cpu_model" in out


def test_cpu_baseline_threads_follow_omp_and_nproc_is_timed(monkeypatch):
    """OMP_NUM_THREADS below nproc: the value runs at OMP_NUM_THREADS (the CPUs
    this process may use), nproc threads are timed beside it."""
    import os
    nproc = len(os.sched_getaffinity(0))
    if nproc < 2:
        pytest.skip("needs 2 CPUs")
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    out = bench.cpu_baseline("cfg2", 8, 1, 1 << 16, 1024, 0.2, None, sample_bytes=16 << 20)
    assert out["cores"] == 1 and out["omp_num_threads"] == 1
    assert set(out["by_threads"]) == {"1", str(nproc)} and "nproc" in out["threads_note"]


def test_cpu_places_prefers_the_gpu_node_and_physical_cores(tmp_path):
    """cpu_places on a made-up two-node sysfs with SMT siblings (c, c + 8)."""
    node = tmp_path / "devices/system/node"
    for n, cpus in ((0, "0-3,8-11"), (1, "4-7,12-15")):
        (node / f"node{n}").mkdir(parents=True)
        (node / f"node{n}" / "cpulist").write_text(cpus + "\n")
    for c in range(16):
        d = tmp_path / f"devices/system/cpu/cpu{c}/topology"
        d.mkdir(parents=True)
        d.joinpath("thread_siblings_list").write_text(f"{c % 8},{c % 8 + 8}\n")
    allowed = set(range(16))
    # no L3 information: one domain, CPUs in order
    assert bench.cpu_places(3, 1, str(tmp_path), allowed) == [4, 5, 6]
    assert bench.cpu_places(6, 1, str(tmp_path), allowed) == [4, 5, 6, 7, 12, 13]
    assert bench.cpu_places(10, 0, str(tmp_path), allowed) == [0, 1, 2, 3, 8, 9, 10, 11, 4, 5]
    assert bench.cpu_places(2, None, str(tmp_path), {9, 2, 1}) == [1, 2]
    assert bench.parse_cpulist("0-2,7\n") == [0, 1, 2, 7]
    # two L3 domains per node (cores {0,1}, {2,3} on node 0; {4,5}, {6,7} on node 1):
    # threads alternate between them before a domain gets its second core
    for c in range(16):
        d = tmp_path / f"devices/system/cpu/cpu{c}/cache/index3"
        d.mkdir(parents=True)
        base = (c % 8) // 2 * 2
        d.joinpath("shared_cpu_list").write_text(f"{base},{base + 1},{base + 8},{base + 9}\n")
    assert bench.cpu_places(4, 0, str(tmp_path), allowed) == [0, 2, 1, 3]
    assert bench.cpu_places(2, 1, str(tmp_path), allowed) == [4, 6]
    assert bench.cpu_places(6, 1, str(tmp_path), allowed) == [4, 6, 5, 7, 12, 14]


def test_erasure_pattern_is_recoverable_and_exact():
    """bench.erasure_pattern: `lost` zero data bytes per stripe, each in its own
    class, parity intact, so every stripe passes is_recoverable
    (xorec_utils.hpp:160-175) and needs recovery."""
    import numpy as np

    import xorec_oracle as xo
    from bench import erasure_pattern
    for k, m, lost, start in [(16, 1, 1, 0), (16, 4, 4, 5), (32, 8, 8, 3), (8, 2, 2, 17),
                              (16, 4, 2, 0)]:
        bm = erasure_pattern(np, 40, k, m, lost, start)
        assert bm.shape == (40, k + m)
        assert (bm[:, k:] == 1).all()
        assert ((bm[:, :k] == 0).sum(axis=1) == lost).all()
        for row in bm:
            zeros = np.flatnonzero(row[:k] == 0)
            assert len(set(zeros % m)) == lost
            assert xo.np_is_recoverable(k, m, row) and xo.np_require_recovery(k, row)


def test_gpu_numa_node_reads_the_pci_function(tmp_path):
    """The host leg records the NUMA node of each rank's GPU (bench.gpu_numa_node)
    from the PCI function in sysfs; a fake sysfs puts it on node 1."""
    from types import SimpleNamespace

    (tmp_path / "bus/pci/devices/0000:c1:00.0").mkdir(parents=True)
    (tmp_path / "bus/pci/devices/0000:c1:00.0/numa_node").write_text("1\n")
    props = SimpleNamespace(pci_domain_id=0, pci_bus_id=0xC1, pci_device_id=0)
    fake_torch = SimpleNamespace(cuda=SimpleNamespace(get_device_properties=lambda d: props))
    assert bench.gpu_numa_node(fake_torch, 0, sysfs=str(tmp_path)) == {"numa_node": 1}
    (tmp_path / "bus/pci/devices/0000:c1:00.0/numa_node").write_text("-1\n")
    assert "skipped" in bench.gpu_numa_node(fake_torch, 0, sysfs=str(tmp_path))
    props.pci_bus_id = 0x05  # no such device
    assert "skipped" in bench.gpu_numa_node(fake_torch, 0, sysfs=str(tmp_path))
