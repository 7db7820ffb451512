"""xec_set_kernel_events (include/xec.h): the next codec call's kernel records
a start and a stop HIP event from its own dispatch (hipExtLaunchKernel), so
bench.py times every kernel without queueing an event packet between kernels.

Checked: the timed kernels still compute the oracle's bytes; the interval is
the kernel's (positive, and no longer than the same launch bracketed by
hipEventRecord packets on either side); a call that launches nothing consumes
the setting, so a later untimed call never records into stale events; the
device-resident decode times its decode kernel, not its check kernel.
"""
from __future__ import annotations

import numpy as np
import pytest

import xorec_oracle as xo

pytestmark = pytest.mark.gpu


def _ev(torch, s):
    e = torch.cuda.Event(enable_timing=True)
    e.record(s)  # torch creates the HIP handle at the first record
    return e


def test_kernel_events_time_the_codec_kernels(gpu, oracle):
    import torch
    S, k, m, bs = 64, 16, 1, 65536
    s = torch.cuda.current_stream()
    d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
    p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
    assert gpu.fill_splitmix64(d, S, k * bs, xo.RANDOM_SEED, s) == 0
    e0, e1, e2, e3 = (_ev(torch, s) for _ in range(4))
    torch.cuda.synchronize()
    # timed encode: same bytes as the oracle, a positive interval
    assert gpu.set_kernel_events(e0, e1) == gpu.Status.SUCCESS
    assert gpu.encode(d, p, S, bs, k, m, s) == 0
    torch.cuda.synchronize()
    ref_d, ref_p = oracle.batch(S, k, m, bs)
    assert np.array_equal(p.cpu().numpy(), ref_p)
    t_kernel = e0.elapsed_time(e1)
    assert t_kernel > 0
    # the same encode between two packet events: never shorter than the kernel
    e2.record(s)
    assert gpu.encode(d, p, S, bs, k, m, s) == 0
    e3.record(s)
    torch.cuda.synchronize()
    assert t_kernel <= e2.elapsed_time(e3) * 1.5 + 0.01
    # timed decode, one lost block per stripe, rebuilt exactly
    h_bm = torch.from_numpy(xo.single_erasure_bitmap(S, k, m)).pin_memory()
    d_bm = h_bm.to("cuda")
    assert gpu.erase(d, p, S, bs, k, m, d_bm, s) == 0
    assert gpu.set_kernel_events(e2, e3) == gpu.Status.SUCCESS
    assert gpu.decode(d, p, S, bs, k, m, h_bm, torch.empty_like(d_bm), s) == 0
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), ref_d)
    assert e2.elapsed_time(e3) > 0


def test_kernel_events_are_consumed_by_the_next_call(gpu):
    import torch
    S, k, m, bs = 32, 8, 1, 65536
    s = torch.cuda.current_stream()
    d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
    p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
    assert gpu.fill_splitmix64(d, S, k * bs, 7, s) == 0
    e0, e1 = _ev(torch, s), _ev(torch, s)  # recorded back to back: ~0 apart
    torch.cuda.synchronize()
    base = e0.elapsed_time(e1)
    h_bm = torch.ones(S * (k + m), dtype=torch.uint8).pin_memory()  # nothing lost
    assert gpu.set_kernel_events(e0, e1) == gpu.Status.SUCCESS
    assert gpu.decode(d, p, S, bs, k, m, h_bm, h_bm.to("cuda"), s) == 0  # launches nothing
    assert gpu.encode(d, p, S, bs, k, m, s) == 0  # not armed any more: records nothing
    torch.cuda.synchronize()
    assert e0.elapsed_time(e1) == base


def test_kernel_events_device_decode_times_the_decode_kernel(gpu, oracle):
    import torch
    S, k, m, bs = 64, 16, 2, 65536
    s = torch.cuda.current_stream()
    d = torch.empty(S * k * bs, dtype=torch.uint8, device="cuda")
    p = torch.empty(S * m * bs, dtype=torch.uint8, device="cuda")
    assert gpu.fill_splitmix64(d, S, k * bs, xo.RANDOM_SEED, s) == 0
    assert gpu.encode(d, p, S, bs, k, m, s) == 0
    ref_d, _ = oracle.batch(S, k, m, bs)
    h_bm = torch.from_numpy(xo.single_erasure_bitmap(S, k, m)).pin_memory()
    d_bm = h_bm.to("cuda")
    assert gpu.erase(d, p, S, bs, k, m, d_bm, s) == 0
    status = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    e0, e1 = _ev(torch, s), _ev(torch, s)
    torch.cuda.synchronize()
    assert gpu.set_kernel_events(e0, e1) == gpu.Status.SUCCESS
    assert gpu.decode_device(d, p, S, bs, k, m, d_bm, status, s) == 0
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    assert np.array_equal(d.cpu().numpy(), ref_d)
    # the decode kernel moves S*(k/m+1)*bs bytes: far longer than the check kernel
    t = e0.elapsed_time(e1)
    assert t > 0
    assert S * (k // m + 1) * bs / (t * 1e-3) / 1e9 < 8000.0, "faster than HBM: not the decode"
