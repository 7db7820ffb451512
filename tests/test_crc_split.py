"""CPU model of the wave-parallel checksum in csrc/xec_validate.hip.

The reference's block checksum (src/utils/utils.cpp:49-57,86-92) is the chain
crc = rotl(crc, 3) + byte over bytes 8..bs-1, seeded with bs.  The device
kernels split that chain across the 64 lanes of a wave: each lane owns 128
contiguous bytes of an 8 KiB window, computes its segment's ones'-complement
Horner sum S (rotl3 is multiplication by 8 mod 2^32-1, and 8^128 == 1 there),
takes the start state W + sum of the S of the lanes before it, runs the true
chain from that start and checks that it ends where the next lane starts.  A
mismatch (a mod-2^32 carry the ones'-complement sum cannot see) makes the
window fall back to a lane-after-lane walk.  This file runs the same
arithmetic in Python against the plain serial chain, including inputs built to
produce carries, so the split is exact before it reaches the GPU.
"""
from __future__ import annotations

import numpy as np
import pytest

from crc_model import M32, SEG, chain, horner, rotl3, serial_crc, split_crc, steer_to_carry


@pytest.mark.parametrize("bs", [512, 4096, 16640, 65536])
def test_split_matches_serial_random(bs):
    rng = np.random.default_rng(bs)
    for _ in range(3):
        blk = rng.integers(0, 256, bs, dtype=np.uint8).tobytes()
        assert split_crc(blk, bs, {}) == serial_crc(blk, bs)


@pytest.mark.parametrize("lane", [0, 5, 62])
def test_split_falls_back_on_a_carry_and_stays_exact(lane):
    bs = 65536
    rng = np.random.default_rng(lane)
    blk = bytearray(rng.integers(0, 256, bs, dtype=np.uint8).tobytes())
    pos = lane * SEG + 100                # inside `lane`'s segment of window 0
    steer_to_carry(blk, bs, pos)
    stats: dict = {}
    assert split_crc(bytes(blk), bs, stats) == serial_crc(bytes(blk), bs)
    assert stats.get("fallback", 0) >= 1


def test_split_no_fallback_without_carries():
    stats: dict = {}
    bs = 32768
    blk = bytes([0xFF]) * bs
    assert split_crc(blk, bs, stats) == serial_crc(blk, bs)
    # a block of zeros never carries: no fallback, identical result
    stats = {}
    blk = bytes(bs)
    assert split_crc(blk, bs, stats) == serial_crc(blk, bs)
    assert stats.get("fallback", 0) == 0


def test_horner_is_chain_mod_ones_complement():
    rng = np.random.default_rng(3)
    seg = rng.integers(0, 256, SEG, dtype=np.uint8).tobytes()
    assert pow(8, SEG, M32) == 1
    for x in (0, 1, 0x12345678, 0xFFFFFFFE, 0xFFFFFFF0):
        # mod 2^32-1 the chain from x is x + S minus one per mod-2^32 carry
        # (each carry weighted by the powers of 8 still to come, like a byte)
        y, carries = x, 0
        for v in seg:
            t = rotl3(y) + v
            carries = (carries * 8 + (t >> 32)) % M32
            y = t & M32
        assert y % M32 == (x + horner(seg) - carries) % M32


@pytest.mark.parametrize("bs,lanes", [(4096, 32), (256, 2), (384, 4), (65536, 64)])
def test_header_folded_into_segment_zero(bs, lanes):
    """The kernel reads the 8 header bytes as zero and starts at rotl(bs, 8):
    exact for any header content, and through a carry steered into the
    header's own segment (bytes 8..127), at every group width it uses."""
    rng = np.random.default_rng(bs + lanes)
    for header in (bytes(8), bytes([0xFF]) * 8, rng.integers(0, 256, 8, dtype=np.uint8).tobytes()):
        blk = bytearray(rng.integers(0, 256, bs, dtype=np.uint8).tobytes())
        blk[:8] = header
        assert split_crc(bytes(blk), bs, {}, lanes) == serial_crc(bytes(blk), bs)
    blk = bytearray(rng.integers(0, 256, bs, dtype=np.uint8).tobytes())
    steer_to_carry(blk, bs, 60)           # a carry inside segment 0, after the header
    stats: dict = {}
    assert split_crc(bytes(blk), bs, stats, lanes) == serial_crc(bytes(blk), bs)
    assert stats.get("fallback", 0) >= 1

