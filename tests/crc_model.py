"""Python model of the device checksum split (csrc/xec_validate.hip), shared by
tests/test_crc_split.py (CPU) and tests/test_gpu_validate.py (GPU inputs that
force the split's fallback).  Test infrastructure only."""
from __future__ import annotations

M32 = 0xFFFFFFFF
LANES, SEG = 64, 128


def rotl3(x: int) -> int:
    return ((x << 3) | (x >> 29)) & M32


def serial_crc(blk: bytes, bs: int) -> int:
    crc = bs & M32
    for v in blk[8:bs]:
        crc = (rotl3(crc) + v) & M32
    return crc


def oc_add(a: int, b: int) -> int:
    s = a + b
    return (s & M32) + (s >> 32)


def chain(x: int, seg: bytes) -> int:
    for v in seg:
        x = (rotl3(x) + v) & M32
    return x


def horner(seg: bytes) -> int:
    s = 0
    for v in seg:
        s = oc_add(rotl3(s), v)
    return s


def rotl8(x: int) -> int:
    return ((x << 8) | (x >> 24)) & M32


def split_crc(blk: bytes, bs: int, stats: dict, lanes: int = LANES) -> int:
    """Mirror of wave_validate_kernel in xec_validate.hip: the block as
    segments of SEG bytes from byte 0, `lanes` per window.  Segment 0's first 8
    bytes (the header) read as zero and the chain starts at rotl(bs, 8): eight
    zero bytes rotate that to bs exactly at byte 8, where the reference chain
    starts (utils.cpp:72-97)."""
    W = rotl8(bs & M32)
    data = bytes(8) + blk[8:bs]
    for base in range(0, bs, lanes * SEG):
        segs = [data[base + j * SEG: base + (j + 1) * SEG] if base + j * SEG < bs else b""
                for j in range(lanes)]
        S = [horner(s) for s in segs]
        starts, acc = [], 0
        for j in range(lanes):
            starts.append(W if j == 0 else oc_add(W, acc))
            acc = oc_add(acc, S[j])
        ends = [chain(starts[j], segs[j]) for j in range(lanes)]
        if all(ends[j] == starts[j + 1] for j in range(lanes - 1)):
            W = ends[-1]
        else:
            stats["fallback"] = stats.get("fallback", 0) + 1
            cur = W
            for j in range(lanes):
                cur = chain(cur, segs[j])
            W = cur
    return W


def steer_to_carry(blk: bytearray, bs: int, pos: int) -> None:
    """Rewrite bytes pos-11..pos-1 so the chain state before byte pos is
    0xFFFFFFFF, then make byte pos nonzero: rotl3 + byte carries out of 32 bits.
    Eleven octal digits of the gap to the target, tried from a few prefixes."""
    for attempt in range(256):
        blk[pos - 12] = attempt
        x = chain(bs & M32, bytes(blk[8:pos - 11]))
        gap = (M32 - ((x << 1 | x >> 31) & M32)) & M32   # 11 rotl3 = rotl 33 = rotl 1
        digits = [(gap >> (3 * (10 - i))) & 7 for i in range(11)]
        blk[pos - 11:pos] = bytes(digits)
        if chain(x, bytes(digits)) == M32:
            blk[pos] = 0x80
            return
    raise AssertionError("could not steer the chain")
