#!/usr/bin/env python3
"""Probe: RCCL batched send-to-self of one message of each size (one GPU,
world 1), bit-exact or not.  Found a 4 GiB + 4 KiB message corrupted with no
error (round 2); xec/dist.py therefore splits every transfer into pieces of
at most xdist.P2P_PIECE_BYTES.  Prints one line per size.

    python tools/rccl/p2p_size_probe.py
"""
import socket
import sys

import torch
import torch.distributed as dist

with socket.socket() as s:
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0),
                        init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
sizes = [int(x) for x in sys.argv[1:]] or [
    64 << 20, 256 << 20, 512 << 20, (1 << 30) - 4096, 1 << 30, (1 << 30) + 4096, 3 << 29,
    (1 << 31) - 4096, 1 << 32]
for n in sizes:
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    src.view(torch.int64)[:n // 8].copy_(torch.arange(n // 8, device="cuda", dtype=torch.int64))
    dst = torch.zeros_like(src)
    ops = [dist.P2POp(dist.isend, src, 0), dist.P2POp(dist.irecv, dst, 0)]
    err = ""
    try:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001
        err = repr(e)[:120]
    ok = (not err) and bool(torch.equal(src, dst))
    first_bad = -1
    if not ok and not err:
        first_bad = int(torch.argmax((src != dst).to(torch.uint8)))
    print(f"bytes={n} ({n / 2**30:.3f} GiB) bit_exact={ok} first_bad_byte={first_bad} {err}",
          flush=True)
    del src, dst
    torch.cuda.empty_cache()
dist.destroy_process_group()
