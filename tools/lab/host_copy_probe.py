#!/usr/bin/env python3
"""How fast can host threads copy pageable memory into pinned memory?

The pipeline stages pageable inputs through pinned buffers filled by a pool of
host threads (csrc/xec_pipeline.cpp HostPool); that only pays if the threads
copy faster than PCIe (~57 GB/s).  This times numpy copies (which release the
GIL, so Python threads run them in parallel) of 1 GiB from pageable into
pinned memory, cut into tasks, at several thread counts -- alone and while a
pinned H2D DMA of the same size runs on the GPU -- and prints the CPU budget
the process has (affinity mask, cgroup quota).

    python tools/lab/host_copy_probe.py [--gib 1] [--threads 1,2,4,8,16] [--task-mib 2,8]
"""
from __future__ import annotations

import argparse
import json
import os
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path


def cgroup_quota():
    try:
        q, p = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--task-mib", default="2,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import numpy as np
    import torch

    n = int(args.gib * (1 << 30))
    src = np.empty(n, np.uint8)
    src[:] = 7  # touched: resident pages, as a caller's filled buffer
    pinned = torch.empty(n, dtype=torch.uint8).pin_memory()
    dst = pinned.numpy()
    pageable_dst = np.empty(n, np.uint8)
    pageable_dst[:] = 0
    dma_src = torch.empty(n, dtype=torch.uint8).pin_memory()
    dev = torch.empty(n, dtype=torch.uint8, device="cuda")
    res = {"bytes": n, "affinity_cpus": len(os.sched_getaffinity(0)),
           "cgroup_quota_cpus": cgroup_quota(), "rows": []}
    print(json.dumps({k: v for k, v in res.items() if k != "rows"}), flush=True)

    def copy(d, t, task):
        def one(o):
            e = min(o + task, n)
            np.copyto(d[o:e], src[o:e])
        with ThreadPoolExecutor(t) as ex:
            list(ex.map(one, range(0, n, task)))

    for task_mib in (int(x) for x in args.task_mib.split(",")):
        task = task_mib << 20
        for t in (int(x) for x in args.threads.split(",")):
            for dname, d in (("pinned", dst), ("pageable", pageable_dst)):
                for with_dma in (False, True):
                    best = None
                    for _ in range(args.reps):
                        torch.cuda.synchronize()
                        if with_dma:
                            dev.copy_(dma_src, non_blocking=True)
                        t0 = time.perf_counter()
                        copy(d, t, task)
                        dt = time.perf_counter() - t0
                        torch.cuda.synchronize()
                        best = dt if best is None else min(best, dt)
                    row = {"task_mib": task_mib, "threads": t, "dst": dname, "dma": with_dma,
                           "GBps": round(n / best / 1e9, 2)}
                    res["rows"].append(row)
                    print(json.dumps(row), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
