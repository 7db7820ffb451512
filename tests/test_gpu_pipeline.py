"""Host-in / host-out pipeline (xec_pipeline_*) on the GPU: bit-exact against the
oracle for encode and erase+decode, ragged last chunk, chunks with no loss."""
from __future__ import annotations

import numpy as np
import pytest


pytestmark = pytest.mark.gpu


def _pinned(nbytes):
    import torch
    return torch.empty(max(nbytes, 1), dtype=torch.uint8).pin_memory()


@pytest.mark.parametrize("S,k,m,bs,chunk,ns,lost", [
    (37, 8, 1, 65536, 8, 2, 1), (256, 16, 1, 1 << 20, 16, 3, 1), (100, 12, 4, 4096, 7, 4, 4),
    (5, 4, 1, 4096, 16, 2, 1), (64, 32, 8, 1024, 1, 1, 8),
    # m > 1 at >= 64 KiB blocks: only the classes that lost a data block travel
    (40, 16, 4, 65536, 8, 3, 1), (24, 16, 4, 65536, 5, 2, 2), (12, 8, 2, 1 << 20, 4, 2, 2),
    (9, 24, 8, 65536, 4, 3, 3),
    # small blocks gather the rebuilt blocks on the device: more than one gather
    # launch per chunk (> 1,024 rebuilt blocks), and k > 256 (per-block copies)
    (3001, 4, 4, 256, 1500, 2, 4), (20, 300, 3, 256, 8, 2, 3),
    # below 1 MiB blocks: selective inputs with gathered outputs, and whole inputs
    (20, 16, 2, 262144, 4, 2, 2), (33, 8, 1, 524288, 4, 3, 1),
])
def test_pipeline_encode_decode(gpu, oracle, S, k, m, bs, chunk, ns, lost):
    ref_d, ref_p = oracle.batch(S, k, m, bs)
    h_d = _pinned(S * k * bs)
    h_p = _pinned(S * m * bs)
    h_d.numpy()[:] = ref_d
    with gpu.Pipeline(chunk, bs, k, m, ns) as pl:
        assert pl.encode(h_d, h_p, S) == gpu.Status.SUCCESS
        assert np.array_equal(h_p.numpy(), ref_p)
        # erase a recoverable set in every other stripe; odd stripes keep all data
        bm = np.ones((S, k + m), np.uint8)
        for c in range(0, S, 2):
            oracle.select_lost_blocks(k, m, lost, bm[c], c)
        d = h_d.numpy().reshape(S, k, bs)
        d[bm[:, :k] == 0] = 0
        h_bm = _pinned(S * (k + m))
        h_bm.numpy()[:] = bm.reshape(-1)
        assert pl.decode(h_d, h_p, S, h_bm) == gpu.Status.SUCCESS
        assert np.array_equal(h_d.numpy(), ref_d)
        assert np.array_equal(h_p.numpy(), ref_p)
        # unrecoverable -> 4, host data untouched
        bm2 = np.ones((S, k + m), np.uint8)
        bm2[0, 0] = 0
        bm2[0, k] = 0
        h_bm.numpy()[:] = bm2.reshape(-1)
        d[0, 0] = 0x11
        assert pl.decode(h_d, h_p, S, h_bm) == gpu.Status.DECODE_FAILURE
        assert (d[0, 0] == 0x11).all()


def test_pipeline_rejects_bad_args(gpu):
    with pytest.raises(RuntimeError):
        gpu.Pipeline(8, 100, 4, 1)
    with pytest.raises(RuntimeError):
        gpu.Pipeline(0, 4096, 4, 1)
    with pytest.raises(RuntimeError):
        gpu.Pipeline(8, 4096, 6, 4)


@pytest.mark.parametrize("ns,lossy_chunks", [(3, [0, 3, 6]), (2, [0, 2, 4, 5]), (3, [1, 2, 7]),
                                             (1, [0, 1, 4])])
@pytest.mark.parametrize("pinned", [True, False])
def test_pipeline_decode_skipped_chunks_and_pageable(gpu, oracle, ns, lossy_chunks, pinned):
    """A chunk's outputs are queued behind the next rebuilding chunk's inputs
    (csrc/xec_pipeline.cpp kDeferOutputs), and chunks without a loss move
    nothing: losses only in chunks that would share a slot if slots went round
    every chunk (0, 3, 6 with 3 slots), so a slot taken over before its
    rebuilt blocks were copied out would show.  Pageable host buffers (plain
    numpy) as well as pinned ones: file and socket buffers are pageable."""
    S, k, m, bs, chunk = 16, 8, 2, 8192, 2
    ref_d, ref_p = oracle.batch(S, k, m, bs, seed_base=4400 + ns)

    def host(a):
        if not pinned:
            return np.ascontiguousarray(a.reshape(-1)).copy()
        t = _pinned(a.size)
        t.numpy()[:] = a.reshape(-1)
        return t

    h_d, h_p = host(ref_d), host(ref_p)
    view = (h_d if not pinned else h_d.numpy()).reshape(S, k, bs)
    with gpu.Pipeline(chunk, bs, k, m, ns) as pl:
        out_p = host(np.zeros_like(ref_p))
        assert pl.encode(h_d, out_p, S) == gpu.Status.SUCCESS
        assert np.array_equal(np.asarray(out_p if not pinned else out_p.numpy()).reshape(-1),
                              ref_p.reshape(-1))
        bm = np.ones((S, k + m), np.uint8)
        for q in lossy_chunks:
            for c in range(q * chunk, (q + 1) * chunk):
                oracle.select_lost_blocks(k, m, 1 + c % m, bm[c], 91 * c + ns)
                bm[c, k:] = 1  # data losses only
                if not (bm[c, :k] == 0).any():
                    bm[c, c % k] = 0
        view[bm[:, :k] == 0] = 0
        h_bm = host(bm)
        assert pl.decode(h_d, h_p, S, h_bm) == gpu.Status.SUCCESS
        got = np.asarray(h_d if not pinned else h_d.numpy()).reshape(-1)
        assert np.array_equal(got, ref_d.reshape(-1))


@pytest.mark.parametrize("threads,opts", [("0", None), ("0", "s"), ("1", None), ("4", None),
                                          ("4", ""), ("4", "a"), ("4", "f"), ("4", "me"),
                                          ("4", "afe"), ("4", "afes"), ("4", "afen"),
                                          ("4", "afe3"), ("2", "afe4"), ("4", "afep"),
                                          ("0", "p")])
@pytest.mark.parametrize("pin_d,pin_p", [(False, False), (False, True), (True, False)])
@pytest.mark.parametrize("S,k,m,bs,chunk,ns", [(37, 8, 1, 65536, 8, 3), (24, 16, 4, 65536, 5, 2),
                                              (30, 12, 4, 4096, 7, 1), (9, 8, 2, 1 << 20, 2, 3)])
def test_pipeline_staged_pageable_inputs(gpu, oracle, monkeypatch, threads, opts, pin_d, pin_p,
                                         S, k, m, bs, chunk, ns):
    """Inputs in pageable memory go through the pinned staging buffers, filled by
    XEC_PIPELINE_COPY_THREADS host threads one chunk ahead (0 = HIP stages them),
    under every XEC_PIPELINE_STAGE_OPTS variant (a: copies alternate over two
    streams, f: first chunk direct, m: the calling thread waits for a buffer,
    e: encode data staged too, s / n: one chunk's input copies in flight at a time
    always / never, a digit: staging buffers, p: pinned inputs alternate too;
    unset = the library default): every mix of
    pinned and pageable data / parity, selective (m > 1, >= 64 KiB) and
    whole-run copies, one to three slots, ragged last chunk."""
    monkeypatch.setenv("XEC_PIPELINE_COPY_THREADS", threads)
    if opts is None:
        monkeypatch.delenv("XEC_PIPELINE_STAGE_OPTS", raising=False)
    else:
        monkeypatch.setenv("XEC_PIPELINE_STAGE_OPTS", opts)
    ref_d, ref_p = oracle.batch(S, k, m, bs, seed_base=5100 + S)

    def host(a, pin):
        if not pin:
            return np.ascontiguousarray(a.reshape(-1)).copy()
        t = _pinned(a.size)
        t.numpy()[:] = a.reshape(-1)
        return t

    def arr(t):
        return np.asarray(t if isinstance(t, np.ndarray) else t.numpy())

    h_d = host(ref_d, pin_d)
    with gpu.Pipeline(chunk, bs, k, m, ns) as pl:
        out_p = host(np.zeros_like(ref_p), pin_p)
        assert pl.encode(h_d, out_p, S) == gpu.Status.SUCCESS
        assert np.array_equal(arr(out_p), ref_p.reshape(-1))
        bm = np.ones((S, k + m), np.uint8)
        for c in range(0, S, 3):  # every third stripe, 1..m data blocks
            oracle.select_lost_blocks(k, m, 1 + c % m, bm[c], 37 * c + 1)
            bm[c, k:] = 1
            if not (bm[c, :k] == 0).any():
                bm[c, c % k] = 0
        arr(h_d).reshape(S, k, bs)[bm[:, :k] == 0] = 0
        h_p = host(ref_p, pin_p)
        assert pl.decode(h_d, h_p, S, host(bm, True)) == gpu.Status.SUCCESS
        assert np.array_equal(arr(h_d), ref_d.reshape(-1))
        assert np.array_equal(arr(h_p), ref_p.reshape(-1))  # parity is read only
