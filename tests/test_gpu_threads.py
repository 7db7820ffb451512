"""Concurrent callers: the reference calls its CPU codec from OpenMP threads on
disjoint stripes (xorec_bm.cpp:27-58); the C ABI must allow the same from
several host threads, each on its own stream (ctypes drops the GIL for the
call).  Every thread's results must be bit-exact against the oracle."""
from __future__ import annotations

import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_threads_on_separate_streams(gpu, oracle):
    import torch

    S, k, m, bs = 6, 8, 2, 8192
    nthreads = 6
    refs = [oracle.batch(S, k, m, bs, seed_base=7000 + 100 * t) for t in range(nthreads)]
    errors: list[str] = []

    def worker(t: int):
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
                p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
                bm = np.ones((S, k + m), np.uint8)
                for c in range(S):
                    oracle.select_lost_blocks(k, m, 1 + (c + t) % m, bm[c], 50 * t + c)
                h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
                d_bm = h_bm.to("cuda", non_blocking=True)
                scratch = torch.empty_like(d_bm)
                for it in range(20):
                    assert gpu.fill_splitmix64(d, S, k * bs, 7000 + 100 * t, s) == 0
                    assert gpu.encode(d, p, S, bs, k, m, s) == 0
                    assert gpu.erase(d, p, S, bs, k, m, d_bm, s) == 0
                    assert gpu.decode(d, p, S, bs, k, m, h_bm, scratch, s) == 0
                s.synchronize()
                ref_d, ref_p = refs[t]
                if not np.array_equal(d.cpu().numpy(), ref_d):
                    errors.append(f"thread {t}: data")
                want_p = ref_p.reshape(S, m, bs).copy()
                want_p[bm[:, k:] == 0] = 0
                if not np.array_equal(p.cpu().numpy().reshape(S, m, bs), want_p):
                    errors.append(f"thread {t}: parity")
        except Exception as e:  # noqa: BLE001 - collected and asserted below
            errors.append(f"thread {t}: {e!r}")

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=300)
    assert not errors, errors
