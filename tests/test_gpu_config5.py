"""Config 5 (BASELINE.json configs[4]: k=16+1, 1 MiB shards, stripe batches
partitioned over the 8 GPUs of one node) at its FULL shape, in every GPU run
(VERDICT r04 item 1).

bin/xec_multi_leg is the exact program bench.py's multi-device leg runs on the
driver's 8-GPU node (host/xec_multi_leg.cpp).  On a one-GPU box the device
list repeats device 0 eight times: eight shards of 256 stripes, each with its
own stream and 4 GiB of data in HBM, plus the root's 34 GiB batch that the
exchange scatters from (copies past the 4 GiB offset) and gathers parity back
to.  What is asserted is what the 8-GPU run depends on:
  * every timed iteration's decode rebuilt every lost block (validate_block,
    /root/reference/src/utils/utils.cpp:72-97, on every shard),
  * the codec returned success on every shard,
  * the gathered parity equals the root's own encode of the whole batch,
    byte for byte (stripe independence, src/algorithms/xorec_bm.cpp:30).
"""
from __future__ import annotations

import json
import subprocess

import pytest

from conftest import PKG_DIR

LEG = PKG_DIR / "bin" / "xec_multi_leg"


@pytest.mark.gpu
def test_config5_full_shape_one_process_leg():
    assert LEG.exists(), "build with make -C erasure-code-benchmark_amd"
    cmd = [str(LEG), "--devices", ",".join(["0"] * 8), "--stripes-per-device", "256",
           "--data", "16", "--parity", "1", "--block", "1M", "--iterations", "3",
           "--warmup", "1", "--scatter-reps", "1"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, p.stdout + p.stderr
    out = json.loads(lines[-1])
    assert p.returncode == 0, out
    assert "error" not in out, out
    assert out["stripes_total"] == 2048 and out["stripes_per_device"] == 256
    assert out["devices"] == [0] * 8 and out["k"] == 16 and out["m"] == 1
    assert out["block_bytes"] == 1 << 20
    assert out["codec_status"] == 0
    assert out["corrupted_iterations"] == 0
    assert out["bit_exact"] is True
    # one lost block per stripe, drawn over all 17 blocks: ~16/17 of them data
    assert 0 < out["lost_data_blocks_per_iteration"] <= 2048
    sc = out["scatter"]
    assert "error" not in sc, sc
    assert sc["gathered_parity_bit_exact_vs_root_encode"] is True
    assert out["encode_GBps"] > 0 and out["decode_GBps"] > 0
