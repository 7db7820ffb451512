"""The C++ XorecBenchmarkHip plugin + BM_generic-style harness (bin/xec_bench):
reference CSV schema, validation-pattern integrity after erase + decode."""
from __future__ import annotations

import csv
import io
import subprocess

import pytest

from conftest import PKG_DIR

BENCH = PKG_DIR / "bin" / "xec_bench"
HEADER = ("name,err_msg,iterations,warmup_iterations,gpu_computation,gpu_blocks,threads_per_block,"
          "message_size_B,block_size_B,EC,lost_blocks,cpu_threads,encode_time_ns,"
          "encode_time_ns_stddev,encode_throughput_Gbps,encode_throughput_Gbps_stddev,"
          "decode_time_ns,decode_time_ns_stddev,decode_throughput_Gbps,"
          "decode_throughput_Gbps_stddev").split(",")


def run(*args, timeout=600):
    return subprocess.run([str(BENCH), *map(str, args)], capture_output=True, text=True,
                          timeout=timeout)


def test_cli_help_and_lost_check():
    assert BENCH.exists(), "build with make -C erasure-code-benchmark_amd"
    assert run("--help").returncode == 0
    r = run("-k", "4", "-m", "1", "-l", "2")
    assert r.returncode == 2 and "parity" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    ("-s", "64M", "-b", "64K", "-k", "8", "-m", "4", "-l", "4", "-i", "3", "-w", "1"),
    ("-s", "8M", "-b", "1K", "-k", "32", "-m", "8", "-l", "0", "-i", "3"),
    ("-s", "32M", "-b", "4K", "-k", "16", "-m", "4", "-l", "2", "-i", "3"),
    ("-s", "1G", "-b", "1M", "-k", "16", "-m", "1", "-l", "1", "-i", "2", "-w", "1"),
    ("-s", "64M", "-b", "8K", "-k", "16", "-m", "4", "-l", "3", "-i", "2", "-V"),
])
def test_harness_rows_clean(args):
    r = run(*args, "-r", "7")
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
