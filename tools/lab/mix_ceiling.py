#!/usr/bin/env python3
"""Single-erasure decode against what its own read and write streams allow
(VERDICT r2 item 5), in one process on one MI355X.

Per shape (k, m, bs, S), one lost data block per stripe (bench.erasure_pattern:
class c mod m, member (7c) mod k/m), on the same three rotating buffer sets and
the same work list, interleaved over rounds (HIP events on the launching
stream):
  decode  the product, xec_decode with work-list tiles (xec_set_decode_tiling(3):
          the list in the scratch, or in the kernel arguments when <= 1,024)
  auto    the product's automatic tiling
  read    tools/lab/mix_kernels.hip MODE 0: only the decode's reads
  write   MODE 1: only the decode's rebuilt-block writes
  lab     MODE 2: the lab's restatement of the decode (fidelity check)
  spread  MODE 3: the same, tiles walked list-entry-fastest (many rebuilt
          blocks written at once instead of the product's few)
  encode  the product's encode of the same batch (reference point)
all at the product's residency for k/m (xec_api.cpp auto_occupancy).  The mix
ceiling is the two streams one after the other: t_read + t_write for the
decode's bytes; `decode_over_ceiling` = (t_read + t_write) / t_decode, > 1 when
the decode overlaps them.  The product decode is checked bit-exact (erase ->
decode == a fresh fill) at the end.

    python tools/lab/mix_ceiling.py [--shapes 16,8,65536,16384:...] [--out f.json]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))

from bench import algorithmic_bytes, erasure_pattern  # noqa: E402

SHAPES = ("16,8,65536,16384:32,8,65536,8192:16,4,65536,16384:16,2,1048576,256:"
          "16,1,1048576,256:8,1,65536,1024:32,1,4096,65536")
AUTO_OCC = {1: 0, 2: 0, 4: 4, 8: 4, 16: 2, 32: 1}  # xec_api.cpp auto_occupancy


def lds_for(waves: int) -> int:
    if waves <= 0 or waves >= 8:
        return 0
    b = (160 * 1024) // (4 * waves)
    b &= ~511
    return min(b, 65536)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=SHAPES)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--sets", type=int, default=3,
                    help="resident buffer sets (rotated); each row also gives every "
                         "variant's median per set (placement, DESIGN.md §3)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import numpy as np
    import torch

    import xec

    L = ctypes.CDLL(str(ROOT / "tools" / "lab" / "libmix.so"))
    L.mix_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                             ctypes.c_uint32, ctypes.c_void_p]
    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    rows = []
    for shape in args.shapes.split(":"):
        k, m, bs, S = (int(x) for x in shape.split(","))
        nm = k // m
        lds = lds_for(AUTO_OCC[nm])
        sets = []
        for s in range(args.sets):
            d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
            p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
            assert xec.fill_splitmix64(d, S, k * bs, 1000 + s * 7919, stream) == 0
            assert xec.encode(d, p, S, bs, k, m, stream) == 0
            sets.append((d, p))
        bm = erasure_pattern(np, S, k, m, 1)
        cs, ids = np.nonzero(bm[:, :k] == 0)
        items = torch.from_numpy(((cs.astype(np.uint32) << 8) | ids.astype(np.uint32))).cuda()
        n_items = int(items.numel())
        h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
        scratch = [torch.empty(S * (k + m), dtype=torch.uint8, device="cuda")
                   for _ in range(args.sets)]
        b_enc, b_dec = algorithmic_bytes(S, k, m, bs)
        b_read = n_items * nm * bs  # k/m - 1 survivors + the class parity
        b_write = n_items * bs
        assert b_read + b_write == b_dec

        def run(v, i):
            d, p = sets[i % args.sets]
            if v == "encode":
                return xec.encode(d, p, S, bs, k, m, stream)
            if v in ("decode", "auto"):
                return xec.decode(d, p, S, bs, k, m, h_bm, scratch[i % args.sets], stream)
            mode = {"read": 0, "write": 1, "lab": 2, "spread": 3}[v]
            return L.mix_launch(mode, d.data_ptr(), p.data_ptr(), items.data_ptr(), n_items,
                                k, m, bs, lds, sp)

        variants = ["decode", "auto", "read", "write", "lab", "spread", "encode"]
        times = {v: [] for v in variants}
        by_set = {v: [[] for _ in range(args.sets)] for v in variants}
        it = 0
        for _ in range(args.rounds):
            for v in variants:
                assert xec.set_decode_tiling(3 if v == "decode" else 0) == 0
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(args.iters)]
                first = it
                for e0, e1 in evs:
                    e0.record(stream)
                    assert run(v, it) == 0, v
                    e1.record(stream)
                    it += 1
                torch.cuda.synchronize()
                times[v] += [a.elapsed_time(b) for a, b in evs]
                for j, (a, b) in enumerate(evs):
                    by_set[v][(first + j) % args.sets].append(a.elapsed_time(b))
        assert xec.set_decode_tiling(0) == 0
        # the product decode, bit-exact on a fresh batch
        d, p = sets[0]
        fresh = torch.empty_like(d)
        assert xec.fill_splitmix64(d, S, k * bs, 1000, stream) == 0
        assert xec.encode(d, p, S, bs, k, m, stream) == 0
        d_bm = h_bm.to("cuda")
        assert xec.erase(d, p, S, bs, k, m, d_bm, stream) == 0
        assert xec.decode(d, p, S, bs, k, m, h_bm, scratch[0], stream) == 0
        assert xec.fill_splitmix64(fresh, S, k * bs, 1000, stream) == 0
        exact = bool(torch.equal(fresh, d))
        med = {v: statistics.median(ts) for v, ts in times.items()}
        ceiling_ms = med["read"] + med["write"]
        row = {"k": k, "m": m, "bs": bs, "S": S, "lost_blocks": n_items, "members": nm,
               "residency_waves_per_simd": AUTO_OCC[nm] or 8, "decode_bit_exact": exact,
               "read_bytes": b_read, "write_bytes": b_write,
               "median_ms": {v: round(t, 4) for v, t in med.items()},
               "read_TBps": round(b_read / med["read"] / 1e9, 3),
               "write_TBps": round(b_write / med["write"] / 1e9, 3),
               "decode_TBps": round(b_dec / med["decode"] / 1e9, 3),
               "auto_TBps": round(b_dec / med["auto"] / 1e9, 3),
               "lab_TBps": round(b_dec / med["lab"] / 1e9, 3),
               "spread_TBps": round(b_dec / med["spread"] / 1e9, 3),
               "encode_TBps": round(b_enc / med["encode"] / 1e9, 3),
               "mix_ceiling_TBps": round(b_dec / ceiling_ms / 1e9, 3),
               "decode_over_ceiling": round(ceiling_ms / med["decode"], 4),
               "auto_over_ceiling": round(ceiling_ms / med["auto"], 4),
               "decode_frac_8TBps": round(b_dec / med["decode"] / 1e9 / 8.0, 4),
               "median_ms_by_set": {v: [round(statistics.median(t), 4) if t else None
                                        for t in by_set[v]] for v in variants}}
        print(json.dumps(row), flush=True)
        rows.append(row)
        del sets, fresh, scratch, items
        torch.cuda.empty_cache()
    if args.out:
        Path(args.out).write_text(json.dumps(rows, indent=1) + "\n")


if __name__ == "__main__":
    main()
