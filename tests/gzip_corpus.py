"""gzip / zlib stream corpus for the inflate parity tests (test data, not the
product).  Streams come from zlib 1.2.11 itself (Python's zlib module is the
system library the reference links) with every deflate strategy, plus
hand-built gzip headers (FEXTRA / FNAME / FCOMMENT / FHCRC) and seeded
mutations: truncations, bit flips, trailing bytes, a second member.

`zlib_truth(data)` is the reference's accept/reject and output:
gzip_compressor::uncompress (compression/internal/gzip_compressor.cc:161-230)
throws exactly when inflate returns Z_DATA_ERROR / Z_NEED_DICT /
Z_STREAM_ERROR / Z_MEM_ERROR and otherwise returns what inflate produced up
to the end of the first member or of the input -- which is what
zlib.decompressobj(15 + 32).decompress() returns (or raises).
"""
from __future__ import annotations

import random
import struct
import zlib


def zlib_truth(data: bytes):
    d = zlib.decompressobj(15 + 32)
    try:
        return d.decompress(data)
    except zlib.error:
        return None


def _payload(rng: random.Random, n: int, kind: int) -> bytes:
    if kind == 0:
        return bytes(rng.getrandbits(8) for _ in range(n))
    if kind == 1:
        alpha = b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789"
        return bytes(alpha[rng.randrange(61)] for _ in range(n))
    if kind == 2:
        out = bytearray()
        i = 0
        while len(out) < n:
            out += b'{"user":%d,"event":"click","ts":%d,"page":"/home"}' % (i % 97, 1600000000000 + i)
            i += 1
        return bytes(out[:n])
    return bytes([rng.randrange(3)]) * n


def deflate_raw(data: bytes, level: int, strategy: int, mem: int = 8) -> bytes:
    c = zlib.compressobj(level, zlib.DEFLATED, -15, mem, strategy)
    return c.compress(data) + c.flush()


def gzip_member(data: bytes, level: int = 6, strategy: int = zlib.Z_DEFAULT_STRATEGY, *, flags: int = 0,
                extra: bytes = b"x" * 5, name: bytes = b"name.txt", comment: bytes = b"hello") -> bytes:
    hdr = bytearray(b"\x1f\x8b\x08" + bytes([flags]) + struct.pack("<I", 1234567) + b"\x00\x03")
    if flags & 4:
        hdr += struct.pack("<H", len(extra)) + extra
    if flags & 8:
        hdr += name + b"\0"
    if flags & 16:
        hdr += comment + b"\0"
    if flags & 2:
        hdr += struct.pack("<H", zlib.crc32(bytes(hdr)) & 0xFFFF)
    return bytes(hdr) + deflate_raw(data, level, strategy) + struct.pack("<II", zlib.crc32(data), len(data) & 0xFFFFFFFF)


def zlib_stream(data: bytes, level: int = 6) -> bytes:
    return zlib.compress(data, level)


STRATEGIES = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED]


def clean_streams(seed: int = 7, count: int = 60, max_len: int = 70000):
    """Well-formed gzip members (and a few zlib streams) of every strategy."""
    rng = random.Random(seed)
    out = []
    for i in range(count):
        n = rng.choice([0, 1, 2, 17, 100, 1000, 5000, rng.randrange(1, max_len)])
        data = _payload(rng, n, i % 4)
        level = rng.choice([0, 1, 6, 9])
        strat = STRATEGIES[i % len(STRATEGIES)]
        if i % 10 == 9:
            out.append(zlib_stream(data, level))
        else:
            out.append(gzip_member(data, level, strat, flags=rng.choice([0, 0, 0, 2, 4, 8, 16, 30])))
    return out


def mutated_streams(seed: int = 11, count: int = 300):
    """Truncations, bit flips, trailing bytes, two members, header damage."""
    rng = random.Random(seed)
    base = clean_streams(seed + 1, 40, 20000)
    out = []
    for i in range(count):
        s = bytearray(rng.choice(base))
        m = i % 6
        if m == 0 and len(s) > 1:
            s = s[: rng.randrange(1, len(s))]
        elif m == 1:
            for _ in range(rng.randrange(1, 4)):
                k = rng.randrange(len(s))
                s[k] ^= 1 << rng.randrange(8)
        elif m == 2:
            s += bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 20)))
        elif m == 3:
            s += rng.choice(base)
        elif m == 4 and len(s) > 12:
            k = rng.randrange(10, len(s))
            s[k] = rng.getrandbits(8)
            s = s[: rng.randrange(k, len(s) + 1)]
        else:
            k = rng.randrange(min(len(s), 12))
            s[k] ^= 1 << rng.randrange(8)
        out.append(bytes(s))
    # hand-made corner cases
    out += [b"\x1f", b"\x1f\x8b", b"\x1f\x8b\x08", b"\x1f\x8b\x09\x00", b"\x1f\x8b\x08\xe0" + b"\0" * 6,
            b"\x78\x9c", b"\x78\x9c\x03\x00", b"\x78\xbb" + b"\0" * 8, b"\x48\x0d" + b"\0" * 8,
            b"\x78\xda\x63\x00\x00\x00\x01\x00\x01", b"\x00\x00", b"\x1f\x8b\x08\x00" + b"\0" * 6 + b"\x07"]
    return out
