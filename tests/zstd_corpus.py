"""zstd frame corpus for the decoder parity tests (test data, not the
product).  Frames come from libzstd 1.4.8 itself (the system library the
reference links) through ctypes: every compression level class, content-size
and checksum flags, window logs, strategies, streaming flushes (block
boundaries), frames without a pledged size; plus seeded mutations aimed at
headers (first 48 bytes) and anywhere: truncations, bit flips, byte
replacements, trailing garbage, concatenated frames.

`ref_decode(b)` is the reference's accept/reject and output: the oracle's
rpo_zstd_uncompress, stream_zstd::do_uncompress's loop
(compression/stream_zstd.cc:152-178) over libzstd."""
from __future__ import annotations

import ctypes as C
import random

_Z = None


class _Buf(C.Structure):
    _fields_ = [("p", C.c_void_p), ("size", C.c_size_t), ("pos", C.c_size_t)]


def _zstd():
    global _Z
    if _Z is None:
        z = C.CDLL("libzstd.so.1")
        z.ZSTD_createCCtx.restype = C.c_void_p
        z.ZSTD_CCtx_setParameter.argtypes = [C.c_void_p, C.c_int, C.c_int]
        z.ZSTD_compressBound.restype = C.c_size_t
        z.ZSTD_compressBound.argtypes = [C.c_size_t]
        z.ZSTD_freeCCtx.argtypes = [C.c_void_p]
        z.ZSTD_compressStream2.argtypes = [C.c_void_p, C.POINTER(_Buf), C.POINTER(_Buf), C.c_int]
        z.ZSTD_compressStream2.restype = C.c_size_t
        z.ZSTD_isError.argtypes = [C.c_size_t]
        z.ZSTD_CCtx_setPledgedSrcSize.argtypes = [C.c_void_p, C.c_ulonglong]
        _Z = z
    return _Z


def frame(data: bytes, level=3, checksum=0, content_size=1, wlog=0, flushes=(), pledged=True, strategy=0) -> bytes:
    z = _zstd()
    cc = z.ZSTD_createCCtx()
    z.ZSTD_CCtx_setParameter(cc, 100, level)
    z.ZSTD_CCtx_setParameter(cc, 201, checksum)
    z.ZSTD_CCtx_setParameter(cc, 200, content_size)
    if wlog:
        z.ZSTD_CCtx_setParameter(cc, 101, wlog)
    if strategy:
        z.ZSTD_CCtx_setParameter(cc, 107, strategy)
    cap = z.ZSTD_compressBound(len(data)) + 1024 + 64 * len(flushes)
    out = C.create_string_buffer(cap)
    src = C.create_string_buffer(bytes(data), len(data) + 1)
    if pledged:
        z.ZSTD_CCtx_setPledgedSrcSize(cc, len(data))
    o = _Buf(C.cast(out, C.c_void_p), cap, 0)
    cuts = sorted(set(c for c in flushes if 0 < c < len(data))) + [len(data)]
    prev = 0
    for c in cuts:
        i = _Buf(C.cast(src, C.c_void_p).value + prev, c - prev, 0)
        mode = 2 if c == len(data) else 1
        while True:
            r = z.ZSTD_compressStream2(cc, C.byref(o), C.byref(i), mode)
            assert not z.ZSTD_isError(r)
            if r == 0 and i.pos == i.size:
                break
        prev = c
    z.ZSTD_freeCCtx(cc)
    return out.raw[: o.pos]


def payload(rng: random.Random, n: int, kind: int) -> bytes:
    if kind == 0:
        return bytes(rng.getrandbits(8) for _ in range(n))
    if kind == 1:
        a = b"abcdefghijklmnopqrstuvwxyz0123456789 .,"
        return bytes(a[rng.randrange(len(a))] for _ in range(n))
    if kind == 2:
        out = bytearray()
        i = 0
        while len(out) < n:
            out += b'{"user":%d,"event":"click","ts":%d,"page":"/home/%d"}' % (i % 97, 1600000000000 + i * 7, i % 13)
            i += 1
        return bytes(out[:n])
    if kind == 3:
        return bytes([rng.randrange(3)]) * n
    words = [b"alpha", b"beta", b"gamma", b"delta", b"epsilon", b"zeta", b"eta", b"theta"]
    out = bytearray()
    while len(out) < n:
        out += rng.choice(words) + b" "
    return bytes(out[:n])


def random_frames(rng: random.Random, count: int, sizes=(0, 1, 5, 40, 300, 1000, 5000, 20000, 70000, 140000, 300000)):
    out = []
    for _ in range(count):
        n = rng.choice(sizes)
        data = payload(rng, n, rng.randrange(5))
        f = frame(data, level=rng.choice([1, 3, 5, 9, 19, -3]), checksum=rng.randrange(2),
                  content_size=rng.randrange(2), wlog=rng.choice([0, 0, 10, 12, 17]),
                  flushes=[rng.randrange(max(1, n)) for _ in range(rng.randrange(4))], pledged=rng.randrange(3) > 0,
                  strategy=rng.choice([0, 0, 1, 2, 6, 9]))
        out.append((data, f))
    return out


def mutations(rng: random.Random, frames, per: int = 6):
    cases = []
    for _, f in frames:
        cases.append(f)
        for _ in range(per):
            b = bytearray(f)
            m = rng.randrange(5)
            if m == 0 and len(b) > 1:
                b = b[: rng.randrange(1, len(b))]
            elif m == 1:
                for _ in range(rng.randrange(1, 4)):
                    i = rng.randrange(min(len(b), 48)) if rng.random() < 0.6 else rng.randrange(len(b))
                    b[i] ^= 1 << rng.randrange(8)
            elif m == 2:
                b += bytes(rng.getrandbits(8) for _ in range(rng.randrange(1, 9)))
            elif m == 3:
                b += rng.choice(frames)[1]
            else:
                i = rng.randrange(min(len(b), 48)) if rng.random() < 0.6 else rng.randrange(len(b))
                b[i] = rng.getrandbits(8)
            cases.append(bytes(b))
    return cases


def ref_decode(b: bytes, cap: int = 1 << 24):
    from oracle import oracle as O
    from redpanda_amd import abi
    rc, out = O.uncompress(abi.CODEC_ZSTD, b, cap)
    return out if rc == 0 else None


def ring_frames(rng: random.Random, count: int):
    """Frames decoded in libzstd's ring-buffer mode (no content size, a 1-2
    KiB window patched into a frame encoded with a 128 KiB window, blocks of at
    most 900 bytes) whose matches reach past the window: some stay inside the
    DCtx's previous ring segment (libzstd's extDict), some land where the
    current segment has already written over it.  [(data, frame)]"""
    out = []
    for _ in range(count):
        base = bytes(rng.getrandbits(8) for _ in range(rng.choice([200, 600, 1500, 3000])))
        parts = []
        for _k in range(rng.randint(8, 40)):
            s = rng.randrange(len(base))
            parts.append(base[s:s + rng.randint(20, 400)])
            if rng.random() < 0.3:
                parts.append(bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 30))))
        data = b"".join(parts)
        step = rng.choice([300, 500, 700, 900])
        f = bytearray(frame(data, level=rng.choice([1, 3, 9]), content_size=0, wlog=17,
                            flushes=list(range(step, len(data), step)), pledged=False))
        assert f[4] & 0x20 == 0 and f[4] >> 6 == 0  # window descriptor at byte 5, no content size
        f[5] = rng.choice([0x00, 0x08])  # W = 1 KiB / 2 KiB
        out.append((data, bytes(f)))
    return out
