"""CPU oracle for the XOR-EC hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this module.  It is the checker for the HIP path in
``erasure-code-benchmark_amd/`` and never part of it.

Two independent restatements of the reference (kenji-k6/erasure-code-benchmark)
live here:

* ``liboracle.so`` (``xorec_oracle.c``) -- plain C + OpenMP, fast enough for the
  full BASELINE sizes and the timed CPU baseline; wrapped by :class:`COracle`.
* :mod:`numpy` functions below (``np_encode``/``np_decode``/...) -- a second,
  deliberately simple restatement for small cases.

Both cite the reference file:line they follow.  Pinning (tests/test_oracle.py):
the SURVEY.md §8(c) known-answer hashes, the reference sources compiled
unmodified into ``oracle/_ref/ref_driver`` (oracle/Makefile), and the fixtures
in ``tests/golden/`` generated from that driver.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"
REF_DRIVER = HERE / "_ref" / "ref_driver"

# XorecResult, src/xorec/xorec_utils.hpp:26-32
SUCCESS, INVALID_SIZE, INVALID_ALIGNMENT, INVALID_COUNTS, DECODE_FAILURE = range(5)
RANDOM_SEED = 1896  # src/utils/utils.hpp:26
FNV_BASIS = 0xCBF29CE484222325
FNV_PRIME = 0x100000001B3
_M64 = (1 << 64) - 1


# --------------------------------------------------------------------------
# numpy restatement (small cases)
# --------------------------------------------------------------------------
def splitmix64_words(seed: int, n: int) -> np.ndarray:
    """First n outputs of splitmix64 from state ``seed``."""
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def make_data(S: int, k: int, bs: int, seed_base: int = RANDOM_SEED) -> np.ndarray:
    """Batch of S stripes (shape (S, k, bs) uint8); stripe c from seed_base + c."""
    out = np.empty((S, k * bs // 8), dtype=np.uint64)
    for c in range(S):
        out[c] = splitmix64_words(seed_base + c, k * bs // 8)
    return out.view(np.uint8).reshape(S, k, bs)


def fnv1a64(buf, h: int = FNV_BASIS) -> int:
    """FNV-1a-64; pure Python, use only for small buffers (or COracle.fnv1a64)."""
    for b in memoryview(np.ascontiguousarray(buf)).cast("B"):
        h = ((h ^ b) * FNV_PRIME) & _M64
    return h


def np_check_args(bs: int, k: int, m: int, data_aligned=True, parity_aligned=True) -> int:
    """xorec_check_args, src/xorec/xorec_utils.hpp:61-86 (order kept)."""
    if not data_aligned or not parity_aligned:
        return INVALID_ALIGNMENT
    if bs < 256 or bs % 256:
        return INVALID_SIZE
    if k < 1 or m < 1 or k % m:
        return INVALID_COUNTS
    return SUCCESS


def np_require_recovery(k: int, bitmap) -> bool:
    """require_recovery, xorec_utils.hpp:144-149 (bit 0 of each data byte)."""
    b = np.asarray(bitmap, dtype=np.uint8)
    return int((b[:k] & 1).sum()) != k


def np_is_recoverable(k: int, m: int, bitmap) -> bool:
    """is_recoverable, xorec_utils.hpp:160-175."""
    b = np.asarray(bitmap, dtype=np.uint8)
    needed = [b[k + j] == 0 for j in range(m)]
    for i in range(k):
        if b[i] == 0:
            if needed[i % m]:
                return False
            needed[i % m] = True
    return True


def np_encode(data: np.ndarray, m: int) -> np.ndarray:
    """xorec_encode, xorec.cpp:24-59, batched: data (S, k, bs) -> parity (S, m, bs)."""
    S, k, bs = data.shape
    parity = data[:, :m, :].copy()
    for i in range(m, k):
        parity[:, i % m, :] ^= data[:, i, :]
    return parity


def np_decode_stripe(data: np.ndarray, parity: np.ndarray, bitmap) -> int:
    """xorec_decode, xorec.cpp:62-111, one stripe in place: data (k, bs), parity (m, bs)."""
    k, bs = data.shape
    m = parity.shape[0]
    rc = np_check_args(bs, k, m)
    if rc:
        return rc
    if not np_require_recovery(k, bitmap):
        return SUCCESS
    if not np_is_recoverable(k, m, bitmap):
        return DECODE_FAILURE
    for i in range(k):
        if bitmap[i]:
            continue
        rec = parity[i % m].copy()
        for j in range(i % m, k, m):
            if j != i:
                rec ^= data[j]
        data[i] = rec
    return SUCCESS


def np_decode_batch_all_or_nothing(data, parity, bitmap) -> int:
    """The GPU plugin's batch contract, xorec_gpu_cmp.cu:57-115 (parity const)."""
    S, k, bs = data.shape
    m = parity.shape[1]
    rows = np.asarray(bitmap, dtype=np.uint8).reshape(S, k + m)
    rc = np_check_args(bs, k, m)
    if rc:
        return rc
    need = False
    for c in range(S):
        if np_require_recovery(k, rows[c]):
            need = True
        if not np_is_recoverable(k, m, rows[c]):
            return DECODE_FAILURE
    if not need:
        return SUCCESS
    for c in range(S):
        np_decode_stripe(data[c], parity[c], rows[c])
    return SUCCESS


class Pcg32:
    """PCGRandom, src/utils/utils.cpp:17-32."""

    def __init__(self, seed: int, seq: int):
        self.state = 0
        self.inc = ((seq << 1) | 1) & _M64
        self.next()
        self.state = (self.state + seed) & _M64
        self.next()

    def next(self) -> int:
        old = self.state
        self.state = (old * 6364136223846793005 + self.inc) & _M64
        xs = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        return ((xs >> rot) | (xs << ((-rot) & 31))) & 0xFFFFFFFF


def np_select_lost_blocks(k: int, m: int, lost: int, bitmap, seed: int) -> int:
    """select_lost_blocks, src/utils/utils.cpp:100-127 with seed RANDOM_SEED + seed."""
    if lost == 0:
        return 0
    if lost > m:
        return -1
    valid = list(range(k + m))
    rng = Pcg32(RANDOM_SEED + seed, 1)
    for _ in range(lost):
        idx = valid[rng.next() % len(valid)]
        bitmap[idx] = 0
        valid = [v for v in valid if v % m != idx % m]
    return 0


def single_erasure_bitmap(S: int, k: int, m: int) -> np.ndarray:
    """Bench/test erasure convention: data block (7c) mod k of
    stripe c is lost; everything else present.  Shape (S*(k+m),) uint8."""
    bm = np.ones((S, k + m), dtype=np.uint8)
    bm[np.arange(S), (7 * np.arange(S)) % k] = 0
    return bm.reshape(-1)


# --------------------------------------------------------------------------
# C restatement (liboracle.so)
# --------------------------------------------------------------------------
class COracle:
    """ctypes wrapper over liboracle.so (oracle/xorec_oracle.c)."""

    def __init__(self, path: os.PathLike | str = LIB_PATH):
        if not Path(path).exists():
            raise FileNotFoundError(f"{path} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(str(path))
        vp, sz, u8p = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p
        L.xo_check_args.argtypes = [vp, vp, sz, sz, sz]
        L.xo_require_recovery.argtypes = [sz, u8p]
        L.xo_is_recoverable.argtypes = [sz, sz, u8p]
        L.xo_encode.argtypes = [vp, vp, sz, sz, sz]
        L.xo_decode.argtypes = [vp, vp, sz, sz, sz, u8p]
        L.xo_encode_batch.argtypes = [vp, vp, sz, sz, sz, sz, ctypes.c_int]
        L.xo_decode_batch.argtypes = [vp, vp, sz, sz, sz, sz, u8p, ctypes.c_int]
        L.xo_decode_batch_all_or_nothing.argtypes = [vp, vp, sz, sz, sz, sz, u8p, ctypes.c_int]
        L.xo_fill_splitmix64.argtypes = [vp, sz, sz, ctypes.c_uint64, ctypes.c_int]
        L.xo_fnv1a64.argtypes = [vp, sz, ctypes.c_uint64]
        L.xo_fnv1a64.restype = ctypes.c_uint64
        L.xo_select_lost_blocks.argtypes = [sz, sz, sz, u8p, ctypes.c_uint64]
        L.xo_write_validation_pattern.argtypes = [vp, sz, ctypes.c_uint64]
        L.xo_validate_block.argtypes = [vp, sz]
        self.L = L

    @staticmethod
    def _p(a) -> int:
        if isinstance(a, np.ndarray):
            return a.ctypes.data
        return int(a)

    # --- host buffers ------------------------------------------------------
    @staticmethod
    def aligned(nbytes: int, align: int = 64) -> np.ndarray:
        raw = np.empty(nbytes + align, dtype=np.uint8)
        off = (-raw.ctypes.data) % align
        return raw[off:off + nbytes]

    def fill(self, buf: np.ndarray, S: int, stripe_bytes: int, seed_base=RANDOM_SEED, threads=0):
        self.L.xo_fill_splitmix64(self._p(buf), S, stripe_bytes, seed_base, threads)

    def fnv1a64(self, buf, h: int = FNV_BASIS) -> int:
        a = np.ascontiguousarray(buf)
        return int(self.L.xo_fnv1a64(a.ctypes.data, a.nbytes, h))

    # --- codec -------------------------------------------------------------
    def check_args(self, data, parity, bs, k, m) -> int:
        return self.L.xo_check_args(self._p(data), self._p(parity), bs, k, m)

    def encode(self, data, parity, bs, k, m) -> int:
        return self.L.xo_encode(self._p(data), self._p(parity), bs, k, m)

    def decode(self, data, parity, bs, k, m, bitmap) -> int:
        return self.L.xo_decode(self._p(data), self._p(parity), bs, k, m, self._p(bitmap))

    def encode_batch(self, data, parity, S, bs, k, m, threads=0) -> int:
        return self.L.xo_encode_batch(self._p(data), self._p(parity), S, bs, k, m, threads)

    def decode_batch(self, data, parity, S, bs, k, m, bitmap, threads=0) -> int:
        return self.L.xo_decode_batch(self._p(data), self._p(parity), S, bs, k, m,
                                      self._p(bitmap), threads)

    def decode_batch_all_or_nothing(self, data, parity, S, bs, k, m, bitmap, threads=0) -> int:
        return self.L.xo_decode_batch_all_or_nothing(self._p(data), self._p(parity), S, bs, k, m,
                                                     self._p(bitmap), threads)

    def require_recovery(self, k, bitmap) -> bool:
        return bool(self.L.xo_require_recovery(k, self._p(bitmap)))

    def is_recoverable(self, k, m, bitmap) -> bool:
        return bool(self.L.xo_is_recoverable(k, m, self._p(bitmap)))

    def select_lost_blocks(self, k, m, lost, bitmap, seed) -> int:
        return self.L.xo_select_lost_blocks(k, m, lost, self._p(bitmap), seed)

    def write_validation_pattern(self, block, nbytes, seed) -> int:
        return self.L.xo_write_validation_pattern(self._p(block), nbytes, seed)

    def validate_block(self, block, nbytes) -> bool:
        return bool(self.L.xo_validate_block(self._p(block), nbytes))

    # --- convenience ---------------------------------------------------------
    def batch(self, S: int, k: int, m: int, bs: int, seed_base=RANDOM_SEED, threads=0):
        """Fresh (data, parity) host batch, data filled, parity encoded."""
        data = self.aligned(S * k * bs)
        parity = self.aligned(S * m * bs)
        self.fill(data, S, k * bs, seed_base, threads)
        rc = self.encode_batch(data, parity, S, bs, k, m, threads)
        if rc:
            raise RuntimeError(f"oracle encode failed rc={rc}")
        return data, parity
