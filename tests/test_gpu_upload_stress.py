"""Concurrent decodes through the library's upload buffers (csrc/xec_api.cpp
upload_begin / upload_end; DESIGN.md §3 *Uploads*).

`xec_decode` copies the bitmap or the work list into device buffers the
library owns, on a copy stream of its own, and reuses a buffer once the kernel
that read it has passed; at most 16 are kept per device, after which a caller
waits for the oldest reader. The buffers are shared by every thread and
stream of the process. This test drives more callers than buffers, each on
its own stream with a different loss pattern every iteration, and never
synchronises between iterations. If a buffer were handed out while a kernel
still read it, that decode would rebuild from another caller's bitmap or list
and the round trip would not come back to the pristine batch.

The reference calls its codec from concurrent OpenMP threads on disjoint
stripes (xorec_bm.cpp:27-58). The check is the size-independent round trip
erase -> decode == pristine, with parity untouched (xorec.cpp:62-111: parity
is const), so it needs no oracle."""
from __future__ import annotations

import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# (k, m, bs, S, iterations, tiling xec_decode must pick, what is uploaded)
SHAPES = {
    # half the stripes lose one block: 2,048 entries > 1,024, sparse -> list tiles, list upload
    "list": (4, 1, 256, 4096, 24, 3),
    # two losses per stripe, one per class -> class tiles, 20 KiB bitmap upload
    "class": (8, 2, 512, 2048, 24, 2),
    # one loss per stripe, bitmap 320 KiB >= 256 KiB -> stripe tiles, copied before the scan
    "stripe_copy_first": (8, 2, 256, 32768, 12, 1),
}
THREADS = 24  # more callers than the library's 16 buffers per device


def pattern(shape: str, k: int, m: int, S: int, it: int) -> np.ndarray:
    """Bitmap (S, k+m) for iteration `it`, data losses only, at most one per class."""
    bm = np.ones((S, k + m), np.uint8)
    c = np.arange(S)
    if shape == "list":
        hit = (c + it) % 2 == 0
        bm[c[hit], ((c * 3 + it) % k)[hit]] = 0
    elif shape == "class":
        r = k // m
        bm[c, m * ((c + it) % r)] = 0          # class 0
        bm[c, m * ((c * 3 + it) % r) + 1] = 0  # class 1
    else:
        bm[c, (c * 5 + it) % k] = 0
    return bm


def test_concurrent_decodes_share_upload_buffers(gpu):
    import torch

    errors: list[str] = []
    tilings: dict[int, set[int]] = {}

    def worker(t: int):
        name = list(SHAPES)[t % len(SHAPES)]
        k, m, bs, S, iters, _ = SHAPES[name]
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            h_bms = [torch.from_numpy(pattern(name, k, m, S, it + t).reshape(-1)).pin_memory()
                     for it in range(iters)]
            with torch.cuda.stream(s):
                d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
                p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
                assert gpu.fill_splitmix64(d, S, k * bs, 91000 + 1000 * t, s) == 0
                assert gpu.encode(d, p, S, bs, k, m, s) == 0
                pristine, p0 = d.clone(), p.clone()
                d_bms = [h.to("cuda", non_blocking=True) for h in h_bms]
                scratch = torch.empty_like(d_bms[0])
                mismatch = []
                seen = set()
                for it in range(iters):
                    assert gpu.erase(d, p, S, bs, k, m, d_bms[it], s) == 0
                    rc = gpu.decode(d, p, S, bs, k, m, h_bms[it], scratch, s)
                    assert rc == 0, f"decode returned {rc!r}"
                    seen.add(gpu.decode_tiling_used())
                    mismatch.append(torch.ne(d, pristine).any())  # queued, no sync
                s.synchronize()
                tilings[t] = seen
                bad = [it for it, x in enumerate(mismatch) if bool(x)]
                if bad:
                    errors.append(f"thread {t} ({name}): iterations {bad} did not restore the batch")
                if not torch.equal(p, p0):
                    errors.append(f"thread {t} ({name}): parity changed")
        except Exception as e:  # noqa: BLE001 - collected and asserted below
            errors.append(f"thread {t} ({name}): {e!r}")

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(THREADS)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in threads), "a worker did not finish"
    assert not errors, errors
    # each shape took the tiling whose upload it is meant to exercise
    for t, seen in tilings.items():
        name = list(SHAPES)[t % len(SHAPES)]
        assert seen == {SHAPES[name][5]}, f"thread {t} ({name}) used tilings {seen}"


def test_concurrent_per_stripe_decodes_and_pipelines(gpu):
    """The other users of the shared host-side state, concurrently: threads
    running xec_decode_per_stripe (pinned list staging + upload buffers, list
    longer than the kernel arguments hold) beside threads each streaming its
    own pipeline over pageable buffers (bounce buffers + helper thread), with
    an unrecoverable stripe in every other per-stripe batch.  Round trips are
    checked against the pristine bytes; per-stripe codes against the pattern."""
    import torch

    errors: list[str] = []

    def per_stripe(t: int):
        k, m, bs, S = 8, 2, 512, 3000
        try:
            torch.cuda.set_device(0)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
                p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
                assert gpu.fill_splitmix64(d, S, k * bs, 77000 + t, s) == 0
                assert gpu.encode(d, p, S, bs, k, m, s) == 0
                pristine, p0 = d.clone(), p.clone()
                for it in range(8):
                    bm = np.ones((S, k + m), np.uint8)
                    c = np.arange(S)
                    bm[c, (c + it + t) % k] = 0  # one data block per stripe: 3,000 entries
                    bad = (it % 2 == 1)
                    if bad:  # stripe 17 loses a data block and its class parity
                        bm[17, :] = 1
                        bm[17, 0] = 0
                        bm[17, k] = 0
                    h_bm = torch.from_numpy(bm.reshape(-1)).pin_memory()
                    d_bm = h_bm.to("cuda", non_blocking=True)
                    codes = np.full(S, 9, np.uint8)
                    assert gpu.erase(d, p, S, bs, k, m, d_bm, s) == 0
                    st = gpu.decode_per_stripe(d, p, S, bs, k, m, h_bm, torch.empty_like(d_bm),
                                               codes, s)
                    s.synchronize()
                    want = np.zeros(S, np.uint8)
                    if bad:
                        want[17] = 4
                    if st != (4 if bad else 0) or not np.array_equal(codes, want):
                        errors.append(f"per-stripe thread {t} it {it}: status {st}")
                        return
                    got = d.view(S, k * bs)
                    ok_rows = torch.ones(S, dtype=torch.bool)
                    if bad:
                        ok_rows[17] = False
                        # the failing stripe is left as erased (its class-0 parity
                        # too): restore it for the next round
                        d.view(S, k * bs)[17].copy_(pristine.view(S, k * bs)[17])
                        p.copy_(p0)
                    if not torch.equal(got[ok_rows], pristine.view(S, k * bs)[ok_rows]):
                        errors.append(f"per-stripe thread {t} it {it}: bytes")
                        return
        except Exception as e:  # noqa: BLE001 - collected and asserted below
            errors.append(f"per-stripe thread {t}: {e!r}")

    def pipeline(t: int):
        k, m, bs, S = 16, 1, 65536, 96
        try:
            torch.cuda.set_device(0)
            d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
            p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
            assert gpu.fill_splitmix64(d, S, k * bs, 88000 + t, torch.cuda.current_stream()) == 0
            assert gpu.encode(d, p, S, bs, k, m, torch.cuda.current_stream()) == 0
            ref_d, ref_p = d.cpu().numpy(), p.cpu().numpy()
            h_d, h_p = ref_d.copy(), np.zeros_like(ref_p)  # pageable
            with gpu.Pipeline(4, bs, k, m, 3) as pl:
                for it in range(4):
                    h_p[:] = 0
                    if pl.encode(h_d, h_p, S) != 0 or not np.array_equal(h_p, ref_p):
                        errors.append(f"pipeline thread {t} it {it}: encode")
                        return
                    bm = np.ones((S, k + m), np.uint8)
                    c = np.arange(S)
                    sel = (c + it) % 3 == 0
                    bm[c[sel], ((c + t) % k)[sel]] = 0
                    h_d.reshape(S, k, bs)[bm[:, :k] == 0] = 0
                    if pl.decode(h_d, h_p, S, bm.reshape(-1).copy()) != 0 or \
                            not np.array_equal(h_d, ref_d):
                        errors.append(f"pipeline thread {t} it {it}: decode")
                        return
        except Exception as e:  # noqa: BLE001 - collected and asserted below
            errors.append(f"pipeline thread {t}: {e!r}")

    threads = [threading.Thread(target=per_stripe, args=(t,)) for t in range(8)]
    threads += [threading.Thread(target=pipeline, args=(t,)) for t in range(4)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in threads), "a worker did not finish"
    assert not errors, errors
