#!/usr/bin/env python3
"""Does WHERE a buffer set lives in HBM change the encode / decode rate?

Allocates --sets independent buffer sets of one workload (torch caching
allocator, one hipMalloc each at these sizes) plus sets carved out of one big
allocation, and times the product encode and decode on each set separately,
interleaved over rounds (HIP events on the launching stream).  A per-set
spread well above the per-launch noise means physical placement, not the
kernel, sets part of the rate.

    python tools/lab/placement_probe.py [--workload cfg3] [--sets 4] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "erasure-code-benchmark_amd"))

from bench import algorithmic_bytes, workload_shape  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3")
    ap.add_argument("--sets", type=int, default=4)
    ap.add_argument("--carved", type=int, default=2, help="sets carved from one allocation")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--alloc", default="torch",
                    help="comma list of allocators for the --sets sets each: torch (caching "
                         "allocator), hipmalloc, contiguous (hipExtMallocWithFlags "
                         "hipDeviceMallocContiguous)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import numpy as np
    import torch

    import xec

    torch.cuda.set_device(0)
    assert xec.init(0) == 0
    k, m, bs, S, _ = workload_shape(args.workload)
    db, pb = S * k * bs, S * m * bs
    s = torch.cuda.current_stream()
    sets = {}
    hip = None
    keep = []

    class Raw:  # a device buffer from the HIP runtime directly (torch's runtime)
        def __init__(self, nbytes, flags):
            import ctypes
            nonlocal hip
            if hip is None:
                hip = ctypes.CDLL("libamdhip64.so")
                hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
                hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p),
                                                      ctypes.c_size_t, ctypes.c_uint]
            ptr = ctypes.c_void_p()
            rc = (hip.hipMalloc(ctypes.byref(ptr), nbytes) if flags is None else
                  hip.hipExtMallocWithFlags(ctypes.byref(ptr), nbytes, flags))
            assert rc == 0 and ptr.value, f"allocation failed ({rc})"
            self.ptr = ptr.value
            keep.append(self)

        def data_ptr(self):
            return self.ptr

    for a in args.alloc.split(","):
        for i in range(args.sets):
            if a == "torch":
                d = torch.empty(db, dtype=torch.uint8, device="cuda")
                p = torch.empty(pb, dtype=torch.uint8, device="cuda")
            else:
                flags = None if a == "hipmalloc" else 0x4  # hipDeviceMallocContiguous
                d, p = Raw(db, flags), Raw(pb, flags)
            sets[f"{'own' if a == 'torch' else a}{i}"] = (d, p)
    if args.carved:
        big = torch.empty(args.carved * (db + pb), dtype=torch.uint8, device="cuda")
        for i in range(args.carved):
            o = i * (db + pb)
            sets[f"carved{i}"] = (big[o:o + db], big[o + db:o + db + pb])
    for i, (d, p) in enumerate(sets.values()):
        assert xec.fill_splitmix64(d, S, k * bs, 1896 + 7919 * i, s) == 0
        assert xec.encode(d, p, S, bs, k, m, s) == 0
    bm = np.ones((S, k + m), np.uint8)
    bm[np.arange(S), (7 * np.arange(S)) % k] = 0
    h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
    scratch = h_bm.to("cuda")
    b_enc, b_dec = algorithmic_bytes(S, k, m, bs)
    torch.cuda.synchronize()

    names = list(sets)

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        assert fn() == 0
        e1.record(s)
        return e0, e1

    # Consecutive launches always touch different sets (round-robin over all
    # of them), so no launch reads what the one before it wrote.
    res = {n: {"enc": [], "dec": []} for n in names}
    for r in range(args.rounds):
        order = names[r % len(names):] + names[:r % len(names)]
        evs = []
        for _ in range(args.iters):
            for n in order:
                d, p = sets[n]
                evs.append((n, "enc", timed(lambda: xec.encode(d, p, S, bs, k, m, s))))
            for n in order:
                d, p = sets[n]
                evs.append((n, "dec", timed(lambda: xec.decode(d, p, S, bs, k, m, h_bm, scratch, s))))
        torch.cuda.synchronize()
        for n, kind, (a, b) in evs:
            res[n][kind].append(a.elapsed_time(b))
    out = {"workload": args.workload, "k": k, "m": m, "bs": bs, "S": S, "sets": {}}
    for n in names:
        d, p = sets[n]
        e, dd = statistics.median(res[n]["enc"]), statistics.median(res[n]["dec"])
        out["sets"][n] = {"data_ptr": hex(d.data_ptr()), "parity_ptr": hex(p.data_ptr()),
                          "enc_ms_med": round(e, 4), "enc_GBps": round(b_enc / e / 1e6, 1),
                          "enc_ms_min": round(min(res[n]["enc"]), 4),
                          "dec_ms_med": round(dd, 4), "dec_GBps": round(b_dec / dd / 1e6, 1),
                          "dec_ms_min": round(min(res[n]["dec"]), 4)}
        print(n, out["sets"][n], flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
