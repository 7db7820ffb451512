"""The C++ XorecBenchmarkHip plugin + BM_generic-style harness (bin/xec_bench):
the reference's CLI contract (benchmark_suite.cpp:102-212), its GPU config
cross product (get_gpu_configs, :252-277 over bm_config.cpp:3-23), the
20-column CSV schema (csv_reporter.cpp:11-99), and validation-payload
integrity after erase + decode."""
from __future__ import annotations

import csv
import io
import subprocess

import pytest

from conftest import PKG_DIR, ROOT, run_tsan

BENCH = PKG_DIR / "bin" / "xec_bench"
HEADER = ("name,err_msg,iterations,warmup_iterations,gpu_computation,gpu_blocks,threads_per_block,"
          "message_size_B,block_size_B,EC,lost_blocks,cpu_threads,encode_time_ns,"
          "encode_time_ns_stddev,encode_throughput_Gbps,encode_throughput_Gbps_stddev,"
          "decode_time_ns,decode_time_ns_stddev,decode_throughput_Gbps,"
          "decode_throughput_Gbps_stddev").split(",")
CONFIG_COLS = ["gpu_computation", "gpu_blocks", "threads_per_block", "message_size_B",
               "block_size_B", "EC", "lost_blocks", "cpu_threads"]


def run(*args, timeout=600, cwd=None):
    return subprocess.run([str(BENCH), *map(str, args)], capture_output=True, text=True,
                          timeout=timeout, cwd=cwd)


def reference_sweep():
    """The cross product get_gpu_configs builds, in its loop order."""
    out = []
    for bs in (1024, 2048, 4096, 8192):
        for total, data in ((12, 8), (20, 16), (24, 16), (36, 32), (40, 32)):
            for lost in (0, 1, 2, 4, 8):
                if lost <= total - data:
                    out.append((8 << 20, bs, f"({total}/{data})", lost))
    return out


def test_cli_contract_errors():
    """Argument checks of parse_args (benchmark_suite.cpp:102-212); nothing runs."""
    assert BENCH.exists(), "build with make -C erasure-code-benchmark_amd"
    assert run("--help").returncode == 0
    r = run("-i", "3")
    assert r.returncode == 1 and "No benchmarks selected" in r.stderr
    r = run("-g", "xorec-hip", "-f", "out.txt")
    assert r.returncode == 1 and ".csv" in r.stderr
    r = run("-g", "xorec-gpu")
    assert r.returncode == 1 and "Invalid GPU algorithm" in r.stderr
    r = run("-c", "xorec", "-g", "xorec-hip")
    assert r.returncode == 1 and "Invalid CPU algorithm" in r.stderr
    r = run("-g", "xorec-hip", "-s", "avx1024")
    assert r.returncode == 1 and "Invalid SIMD version" in r.stderr
    r = run("-g", "xorec-hip", "-i", "0")
    assert r.returncode == 1 and "iterations" in r.stderr
    r = run("-g", "xorec-hip", "-w", "-1")
    assert r.returncode == 1 and "warmup" in r.stderr
    r = run("-g", "xorec-hip", "--data", "4", "--parity", "1", "--lost", "2")
    assert r.returncode == 2 and "parity" in r.stderr
    r = run("-g", "xorec-hip-multi", "--devices", "0,x")
    assert r.returncode == 1 and "Invalid device" in r.stderr
    r = run("-g", "xorec-hip-multi", "--devices", "0,-1")
    assert r.returncode == 1 and "Invalid device" in r.stderr


def test_csv_location_contract(tmp_path):
    """A bare -f name lands in ../results/raw/ as in the reference (RAW_DIR +
    OUTPUT_FILE, benchmark_suite.cpp:27,346; scripts/utils/data.py reads it
    there); --raw-dir moves it; a path with '/' is used as given.  The CSV is
    opened, with its header, before any device work, so this runs on the CPU
    (the run itself then stops at xec_init without a GPU)."""
    cwd = tmp_path / "a" / "b"
    cwd.mkdir(parents=True)
    cfg = ("--message", "8M", "--block", "4K", "--data", "8", "--parity", "1", "--lost", "0",
           "-i", "1")
    run("-g", "xorec-hip", "-f", "bare.csv", *cfg, cwd=cwd, timeout=120)
    assert (tmp_path / "a" / "results" / "raw" / "bare.csv").read_text().startswith("name,err_msg")
    run("-g", "xorec-hip", "-f", "moved.csv", "--raw-dir", str(tmp_path / "r"), *cfg, cwd=cwd,
        timeout=120)
    assert (tmp_path / "r" / "moved.csv").exists()
    run("-g", "xorec-hip", "-f", "./here.csv", *cfg, cwd=cwd, timeout=120)
    assert (cwd / "here.csv").exists()


@pytest.mark.gpu
def test_reference_gpu_sweep(tmp_path):
    """`xec_bench -g xorec-hip -f out.csv -i 3`: one clean row per config of the
    reference's GPU cross product, in its order; config columns equal the
    reference's own GPU rows where those exist (tools/reference_gpu_rows.csv,
    the "XOR-EC (GPU Computation)" rows of results/raw/final_results.csv);
    -a appends without a header."""
    out = tmp_path / "out.csv"
    r = run("-g", "xorec-hip", "-f", out, "-i", "3", "-s", "avx2,avx512", timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    rows = list(csv.reader(out.open()))
    assert rows[0] == HEADER
    got = [dict(zip(HEADER, x)) for x in rows[1:]]
    want = reference_sweep()
    assert [(int(g["message_size_B"]), int(g["block_size_B"]), g["EC"], int(g["lost_blocks"]))
            for g in got] == want
    for g in got:
        assert g["err_msg"] == "", g
        assert g["iterations"] == "3" and g["warmup_iterations"] == "0"
        assert float(g["encode_throughput_Gbps"]) > 0
    ref = [x for x in csv.DictReader(line for line in
                                     (ROOT / "tools" / "reference_gpu_rows.csv").open()
                                     if not line.startswith("#"))]
    by_cfg = {(g["message_size_B"], g["block_size_B"], g["EC"], g["lost_blocks"]): g for g in got}
    matched = 0
    for x in ref:
        key = (x["message_size_B"], x["block_size_B"], x["EC"].strip('"'), x["lost_blocks"])
        if key in by_cfg:
            matched += 1
            assert [by_cfg[key][c] for c in CONFIG_COLS] == \
                [x[c].strip('"') for c in CONFIG_COLS], key
    assert matched >= 20
    # -a: rows appended, no second header
    r = run("-g", "xorec-hip", "-f", out, "-a", "-i", "2", "--block", "4K", "--data", "16",
            "--parity", "4", "--lost", "2", "--message", "8M", timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rows2 = list(csv.reader(out.open()))
    assert len(rows2) == len(rows) + 1 and rows2[:len(rows)] == rows
    # without -a the file is overwritten
    r = run("-g", "xorec-hip", "-f", out, "-i", "2", "--block", "4K", "--data", "16",
            "--parity", "4", "--lost", "2", "--message", "8M", timeout=300)
    assert r.returncode == 0
    assert len(list(csv.reader(out.open()))) == 2


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    ("--message", "64M", "--block", "64K", "--data", "8", "--parity", "4", "--lost", "4",
     "-i", "3", "-w", "1"),
    ("--message", "8M", "--block", "1K", "--data", "32", "--parity", "8", "--lost", "0", "-i", "3"),
    ("--message", "32M", "--block", "4K", "--data", "16", "--parity", "4", "--lost", "2", "-i", "3"),
    ("--message", "1G", "--block", "1M", "--data", "16", "--parity", "1", "--lost", "1", "-i", "2",
     "-w", "1"),
    ("--message", "64M", "--block", "8K", "--data", "16", "--parity", "4", "--lost", "3", "-i", "2",
     "--host-validation"),
])
def test_harness_rows_clean(args):
    r = run("-g", "xorec-hip", "--stdout", *args, "--seed", "7")
    assert r.returncode == 0, r.stderr + r.stdout
    rows = list(csv.reader(io.StringIO(r.stdout)))
    assert rows[0] == HEADER
    row = dict(zip(HEADER, rows[1]))
    assert row["err_msg"] == ""
    assert row["name"] == "XOR-EC (HIP gfx950)"
    assert float(row["encode_throughput_Gbps"]) > 0
    lost = int(row["lost_blocks"])
    if lost:
        assert float(row["decode_throughput_Gbps"]) > 0


MULTI_EQUIV = ROOT / "tests" / "host" / "bin" / "multi_equiv"


@pytest.mark.gpu
def test_multi_device_plugin_matches_single_device():
    """XorecBenchmarkHipMulti over device lists that repeat device 0 (2-4
    stripe ranges with their own streams and buffers, uneven and empty ranges)
    gives the one-device plugin's bytes after encode, erasure and decode
    (tests/host/multi_equiv.cpp, built by __graft_entry__.build())."""
    assert MULTI_EQUIV.exists(), "build with make -C tests/host"
    p = subprocess.run([str(MULTI_EQUIV)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "multi_equiv ok" in p.stdout, p.stdout + p.stderr


MULTI_SCATTER = ROOT / "tests" / "host" / "bin" / "multi_scatter"


@pytest.mark.gpu
def test_multi_device_scatter_gather():
    """Config 5's exchange in one process: a batch in device 0's HBM scattered
    over the shards with peer copies, encoded per shard, parity gathered back
    == device 0's own encode; shard data == its range of the root batch
    (tests/host/multi_scatter.cpp; ragged, empty and single ranges)."""
    assert MULTI_SCATTER.exists(), "build with make -C tests/host"
    p = subprocess.run([str(MULTI_SCATTER)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "multi_scatter ok" in p.stdout, p.stdout + p.stderr


@pytest.mark.gpu
def test_multi_device_scatter_gather_distinct_gpus():
    """The same exchange over the distinct devices 0 .. min(n, 8) - 1 (VERDICT
    r05 item 1): peer copies between GPUs, 4.5 GiB ones included, and every
    remote shard reached the root by peer access, not a staged copy
    (multi_scatter --distinct).  Skipped on a one-GPU box."""
    import torch
    n = torch.cuda.device_count()  # counts devices without initialising one
    if n < 2:
        pytest.skip(f"{n} GPU visible: peer copies between distinct GPUs need 2 or more")
    assert MULTI_SCATTER.exists(), "build with make -C tests/host"
    p = subprocess.run([str(MULTI_SCATTER), "--distinct"], capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0 and "multi_scatter ok" in p.stdout, p.stdout + p.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("prog,ok", [("asan_multi_equiv", "multi_equiv ok"),
                                     ("asan_multi_scatter", "multi_scatter ok"),
                                     ("asan_abi", "abi_asan ok")])
def test_plugins_under_asan(prog, ok):
    """Host code under AddressSanitizer on the GPU box: both plugins (buffers,
    shards, per-shard decode threads, peer copies) and the C ABI itself (scans,
    work-list staging, kernel-argument lists, per-stripe decode, pipeline run
    merging, over exact-size host buffers; tests/host/abi_asan.cpp).  The host
    side only is instrumented (tests/host/Makefile bin/asan_*); any report
    fails the run."""
    import os
    exe = ROOT / "tests" / "host" / "bin" / prog
    assert exe.exists(), "build with make -C tests/host"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0:"
                                        "abort_on_error=0:exitcode=23")
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0 and ok in p.stdout, p.stdout[-2000:] + p.stderr[-4000:]
    assert "AddressSanitizer" not in p.stderr, p.stderr[-4000:]


@pytest.mark.gpu
def test_overrides_per_thread_under_tsan():
    """Tuning overrides are per thread (include/xec.h): three threads with
    different xec_set_launch / xec_set_occupancy / xec_set_decode_tiling /
    xec_set_validate_kernel settings run encode -> erase -> decode -> validate
    concurrently, each sees only its own tiling and gets exact bytes, and the
    C ABI's host code runs under ThreadSanitizer (tests/host/tsan_overrides.cpp;
    host side only instrumented).  Any race report fails the run."""
    import os
    exe = ROOT / "tests" / "host" / "bin" / "tsan_overrides"
    assert exe.exists(), "build with make -C tests/host"
    supp = ROOT / "tests" / "host" / "tsan.supp"  # HSA-internal new/delete only
    env = dict(os.environ, TSAN_OPTIONS=f"exitcode=23:halt_on_error=0:suppressions={supp}")
    p = run_tsan([str(exe)], timeout=300, env=env)
    assert "ThreadSanitizer" not in p.stderr, p.stderr[-6000:]
    assert p.returncode == 0 and "tsan_overrides ok" in p.stdout, p.stdout[-2000:] + p.stderr[-4000:]


@pytest.mark.gpu
def test_multi_device_rows_clean():
    """`-g xorec-hip,xorec-hip-multi --devices 0,0,0`: one clean row per
    algorithm, in -g order (get_benchmarks, benchmark_suite.cpp:279-311); the
    multi-device run validates every block after erase + decode."""
    r = run("-g", "xorec-hip,xorec-hip-multi", "--devices", "0,0,0", "--stdout", "--message", "64M",
            "--block", "64K", "--data", "8", "--parity", "4", "--lost", "4", "-i", "3", "-w", "1",
            "--seed", "3")
    assert r.returncode == 0, r.stderr + r.stdout
    rows = [dict(zip(HEADER, x)) for x in list(csv.reader(io.StringIO(r.stdout)))[1:]]
    assert [x["name"] for x in rows] == ["XOR-EC (HIP gfx950)",
                                         "XOR-EC (HIP gfx950, multi-device)"]
    for x in rows:
        assert x["err_msg"] == "", x
        assert float(x["encode_throughput_Gbps"]) > 0 and float(x["decode_throughput_Gbps"]) > 0
