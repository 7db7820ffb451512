#!/usr/bin/env python3
"""Child process of tests/test_gpu_parity.py::test_decode_scratch_upload_fallback.

Run with XEC_SCRATCH_UPLOADS=1: xec_decode / xec_decode_per_stripe then copy
their bitmap or work list into the caller's scratch on the stream (the path
taken when no library device buffer can be had).  Every case is erase -> decode
on the GPU, compared with the oracle's batch (the checker).  Prints
"scratch uploads ok".
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "erasure-code-benchmark_amd", ROOT / "oracle"):
    sys.path.insert(0, str(p))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import xec  # noqa: E402
import xorec_oracle as xo  # noqa: E402


def main():
    assert os.environ.get("XEC_SCRATCH_UPLOADS") == "1"
    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    o = xo.COracle()
    s = torch.cuda.current_stream()
    rng = np.random.default_rng(11)
    # (S, k, m, bs, pattern, tiling, per_stripe)
    cases = [
        (2048, 4, 1, 256, "every", 0, False),    # stripe tiles: bitmap via the scratch
        (18432, 4, 1, 256, "sparse", 0, False),  # 2,048-entry list via the scratch
        (1040, 16, 2, 1024, "every_class", 0, False),  # class tiles (past the argument masks)
        (300, 16, 4, 1024, "every_class", 3, False),  # forced list of 1,200 > 1,024 entries
        (5000, 8, 8, 256, "every_class", 0, True),    # per-stripe: list in pieces
        (4096, 4, 2, 256, "every_class", 0, True),
    ]
    for S, k, m, bs, pattern, tiling, per_stripe in cases:
        d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
        p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
        assert xec.fill_splitmix64(d, S, k * bs, xo.RANDOM_SEED, s) == 0
        assert xec.encode(d, p, S, bs, k, m, s) == 0
        ref_d, ref_p = o.batch(S, k, m, bs)
        bm = np.ones((S, k + m), np.uint8)
        for c in range(S):
            if pattern == "every" or (pattern == "sparse" and c % 9 == 4):
                bm[c, (7 * c) % k] = 0
            elif pattern == "every_class":
                for j in range(m):
                    bm[c, j + m * int(rng.integers(k // m))] = 0
        h_bm = torch.from_numpy(bm.reshape(-1).copy()).pin_memory()
        d_bm = h_bm.to("cuda")
        scratch = torch.empty_like(d_bm)
        assert xec.erase(d, p, S, bs, k, m, d_bm, s) == 0
        assert xec.set_decode_tiling(tiling) == 0
        if per_stripe:
            codes = np.full(S, 0xAA, np.uint8)
            st = xec.decode_per_stripe(d, p, S, bs, k, m, h_bm, scratch, codes, s)
            assert codes.tolist() == [0] * S, (S, k, m)
        else:
            st = xec.decode(d, p, S, bs, k, m, h_bm, scratch, s)
        assert xec.set_decode_tiling(0) == 0
        assert st == 0, (S, k, m, bs, pattern, st)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy(), ref_d), (S, k, m, bs, pattern)
        assert np.array_equal(p.cpu().numpy(), ref_p), "decode wrote parity"
        print(f"ok S={S} k={k}+{m} bs={bs} {pattern} tiling={tiling} "
              f"used={xec.decode_tiling_used()}", flush=True)
    print("scratch uploads ok")


if __name__ == "__main__":
    main()
