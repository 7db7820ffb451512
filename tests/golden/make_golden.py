#!/usr/bin/env python3
"""Generate tests/golden/ fixtures from the REFERENCE itself.

Runs oracle/_ref/ref_driver -- the reference's own src/xorec + src/utils
sources compiled unmodified by `make -C oracle ref` -- and records its outputs
as data: known-answer parity hashes, decode results and status codes, plus the
raw parity of BASELINE config 1 and the erasure patterns used.

Only runnable where /root/reference exists (this container); the fixtures it
writes are committed and travel to the GPU box, the driver does not need to.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "oracle"))
import xorec_oracle as xo  # noqa: E402  (generates erasure patterns only)

DRIVER = ROOT / "oracle" / "_ref" / "ref_driver"
OUT = Path(__file__).resolve().parent
SEED = xo.RANDOM_SEED

# (k, m, bs, S): every BASELINE.json config shape at 1-stripe / small-S size,
# the reference's own sweep shapes (bm_config.cpp:3-23: (12/8),(20/16),(24/16),
# (36/32),(40/32) at 1-8 KiB), and edge shapes (k=m, generic member counts,
# minimum block, blocks that are not a multiple of one 4 KiB tile).
ENC_CASES = [
    (4, 1, 4096, 1), (8, 1, 65536, 1), (16, 1, 1048576, 1), (32, 1, 4096, 1), (8, 4, 1024, 1),
    (8, 1, 65536, 16), (16, 1, 1048576, 4), (32, 1, 4096, 64), (4, 1, 4096, 7),
    (8, 4, 1024, 8), (16, 4, 4096, 8), (16, 8, 2048, 8), (32, 4, 8192, 4), (32, 8, 1024, 16),
    (1, 1, 256, 3), (2, 2, 512, 3), (5, 1, 768, 3), (64, 1, 256, 2), (40, 8, 4352, 3),
    (6, 3, 512, 5), (3, 1, 256, 1),
]

# decode cases: (k, m, bs, S, mode, lost_per_stripe)
DEC_CASES = [
    (4, 1, 4096, 1, "single7", 1), (16, 1, 1048576, 4, "single7", 1), (32, 1, 4096, 64, "single7", 1),
    (8, 1, 65536, 8, "single7", 1),
    (8, 4, 1024, 8, "select", 4), (16, 4, 4096, 8, "select", 2), (32, 8, 1024, 16, "select", 8),
    (40, 8, 4352, 3, "select", 5), (5, 1, 768, 3, "select", 1), (64, 1, 256, 2, "select", 1),
    (2, 2, 512, 3, "select", 2),
    (8, 4, 1024, 4, "parity_only", 0), (8, 4, 1024, 4, "none", 0), (8, 4, 1024, 4, "double", 0),
    (16, 1, 4096, 4, "data_and_parity", 0), (8, 1, 1024, 3, "even_byte", 0),
]

# status cases: (k, m, bs, data_misalign, parity_misalign)
CHK_CASES = [
    (4, 1, 100, 0, 0), (4, 1, 4096, 8, 0), (4, 1, 4096, 0, 32), (4, 1, 4096, 0, 0),
    (6, 4, 4096, 0, 0), (4, 0, 4096, 0, 0), (0, 1, 4096, 0, 0), (4, 1, 256, 0, 0),
    (4, 1, 320, 0, 0), (4, 1, 255, 0, 0), (1, 1, 256, 0, 0), (4, 1, 100, 8, 0),
    (6, 4, 100, 0, 0),
]


def run(*args) -> dict:
    out = subprocess.run([str(DRIVER), *map(str, args)], check=True, capture_output=True,
                         text=True).stdout
    return dict(line.split(" ", 1) for line in out.strip().splitlines())


def make_pattern(k, m, S, mode, lost) -> np.ndarray:
    bm = np.ones((S, k + m), dtype=np.uint8)
    if mode == "single7":
        return xo.single_erasure_bitmap(S, k, m).reshape(S, k + m)
    if mode == "select":
        for c in range(S):
            assert xo.np_select_lost_blocks(k, m, lost, bm[c], seed=1000 + c) == 0
    elif mode == "parity_only":
        bm[:, k:] = 0
    elif mode == "double":  # stripe 1 loses two data blocks of class 0 -> DecodeFailure
        bm[0, 1] = 0
        bm[1, 0] = 0
        bm[1, m] = 0
    elif mode == "data_and_parity":  # stripe 2: data block and its parity both lost
        bm[0, 3] = 0
        bm[2, 5] = 0
        bm[2, k + 5 % m] = 0
    elif mode == "even_byte":  # nonzero bytes with bit 0 clear (require_recovery quirk)
        bm[0, 2] = 2
        bm[1, 0] = 0
        bm[2, 1] = 4
    return bm


def main() -> None:
    if not DRIVER.exists():
        sys.exit(f"{DRIVER} missing: run `make -C oracle ref` (needs /root/reference)")
    ka = {"generator": "oracle/_ref/ref_driver (reference src/xorec, src/utils, unmodified)",
          "data": "stripe c = little-endian u64 splitmix64 outputs from state seed+c",
          "seed": SEED, "hash": "FNV-1a-64", "encode": [], "decode": [], "status": []}
    for (k, m, bs, S) in ENC_CASES:
        hashes = {run("enc", k, m, bs, S, SEED, v)["parity_fnv"] for v in range(4)}
        assert len(hashes) == 1, f"reference versions disagree on {(k, m, bs, S)}"
        ka["encode"].append({"k": k, "m": m, "bs": bs, "S": S, "parity_fnv": hashes.pop()})
    pat_dir = OUT / "patterns"
    pat_dir.mkdir(exist_ok=True)
    for (k, m, bs, S, mode, lost) in DEC_CASES:
        bm = make_pattern(k, m, S, mode, lost)
        name = f"bm_k{k}_m{m}_S{S}_{mode}.bin"
        (pat_dir / name).write_bytes(bm.tobytes())
        r = run("dec", k, m, bs, S, SEED, 3, "pattern", pat_dir / name)
        ka["decode"].append({"k": k, "m": m, "bs": bs, "S": S, "mode": mode, "pattern": name,
                             **{key: r[key] for key in ("data_fnv_before", "data_fnv_after",
                                                        "parity_fnv_erased", "parity_fnv_after",
                                                        "codes")}})
    for (k, m, bs, dm, pm) in CHK_CASES:
        r = run("chk", k, m, bs, dm, pm)
        ka["status"].append({"k": k, "m": m, "bs": bs, "data_misalign": dm, "parity_misalign": pm,
                             "encode": int(r["encode"]), "decode": int(r["decode"])})
    # validation pattern: blocks written by the restatement, judged by the
    # reference's validate_block (utils.cpp:72-97); the last block is corrupted.
    lib = xo.COracle()
    blocks = []
    for bs, seed in ((4096, 1), (1024, 2), (8, 3), (256, 4)):
        b = np.zeros(bs, dtype=np.uint8)
        lib.write_validation_pattern(b, bs, seed)
        blocks.append((bs, b))
    bad = blocks[0][1].copy()
    bad[100] ^= 1
    blocks.append((4096, bad))
    ka["validate"] = []
    for i, (bs, b) in enumerate(blocks):
        f = pat_dir / f"val_{i}.bin"
        f.write_bytes(b.tobytes())
        ka["validate"].append({"bs": bs, "file": f.name, "valid": run("val", bs, f)["valid"] == "1"})
    # raw parity for BASELINE config 1 (k=4+1, 4 KiB, one stripe)
    run("enc", 4, 1, 4096, 1, SEED, 3, OUT / "cfg1_parity_k4_m1_4096.bin")
    (OUT / "known_answers.json").write_text(json.dumps(ka, indent=1) + "\n")
    print(f"wrote {OUT / 'known_answers.json'}: {len(ka['encode'])} enc, {len(ka['decode'])} dec, "
          f"{len(ka['status'])} status, {len(ka['validate'])} validate")


if __name__ == "__main__":
    main()
