"""gzip / zstd behind compression::compressor::uncompress: the CPU fallback
of SURVEY.md §8(b) (rpgpu_uncompress with RPGPU_CODEC_GZIP / _ZSTD runs the
reference's own loops over zlib / libzstd on the host, rp_hostcodec.cpp).

Parity: the reference pins no gzip/zstd vectors; the loops are checked against
Python's zlib module (an independent driver of the same library:
gzip_compressor.cc:161-230 semantics — first member only, trailing bytes
ignored, a truncated stream gives what inflated, a data error throws) and
libzstd's one-shot ZSTD_decompress for well-formed frames
(stream_zstd.cc:152-178: frames concatenate, trailing garbage throws).
No GPU needed (ctx may be NULL for these codecs); a GPU test runs the same
cases through a device context and the batch entry point.
"""
import ctypes as C
import gzip
import zlib

import numpy as np
import pytest

from redpanda_amd import abi

_zstd = None


def zstd_lib():
    global _zstd
    if _zstd is None:
        L = C.CDLL("libzstd.so.1")
        L.ZSTD_compress.restype = C.c_size_t
        L.ZSTD_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int]
        L.ZSTD_compressBound.restype = C.c_size_t
        L.ZSTD_compressBound.argtypes = [C.c_size_t]
        L.ZSTD_decompress.restype = C.c_size_t
        L.ZSTD_decompress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.ZSTD_isError.restype = C.c_uint
        L.ZSTD_isError.argtypes = [C.c_size_t]
        _zstd = L
    return _zstd


def zstd_compress(data: bytes, level: int = 3) -> bytes:
    L = zstd_lib()
    cap = L.ZSTD_compressBound(len(data))
    out = C.create_string_buffer(cap)
    n = L.ZSTD_compress(out, cap, data, len(data), level)
    assert not L.ZSTD_isError(n)
    return out.raw[:n]


def uncompress(rplib, codec, payload: bytes, cap: int = 1 << 24, ctx=None):
    L = rplib.load()
    src = np.frombuffer(payload, dtype=np.uint8) if payload else np.zeros(1, dtype=np.uint8)
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    n = C.c_size_t(0)
    rc = L.rpgpu_uncompress(ctx, codec, src.ctypes.data_as(C.c_void_p), len(payload), out.ctypes.data_as(C.c_void_p),
                            cap, C.byref(n))
    return rc, (out[: n.value].tobytes() if rc == 0 else n.value)


def corpus(seed=0, n=300_000):
    rng = np.random.default_rng(seed)
    words = [bytes(rng.integers(97, 123, rng.integers(2, 9), dtype=np.uint8)) for _ in range(200)]
    return b" ".join(words[i] for i in rng.integers(0, len(words), n // 5))[:n]


GZIP_CASES = {
    "text": lambda: (gzip.compress(corpus(1)), corpus(1)),
    "random": lambda: (gzip.compress(bytes(np.random.default_rng(2).integers(0, 256, 100_000, dtype=np.uint8))),
                       bytes(np.random.default_rng(2).integers(0, 256, 100_000, dtype=np.uint8))),
    "zlib_wrapper": lambda: (zlib.compress(corpus(3)), corpus(3)),  # inflateInit2(15 + 32) auto-detects
    "empty_content": lambda: (gzip.compress(b""), b""),
    "second_member_ignored": lambda: (gzip.compress(b"first") + gzip.compress(b"second"), b"first"),
    "trailing_garbage_ignored": lambda: (gzip.compress(corpus(4, 5000)) + b"\x00garbage", corpus(4, 5000)),
}


@pytest.mark.parametrize("name", sorted(GZIP_CASES))
def test_gzip_host_fallback(rplib, name):
    payload, want = GZIP_CASES[name]()
    rc, got = uncompress(rplib, abi.CODEC_GZIP, payload)
    assert rc == 0 and got == want
    # Python's zlib driving the same library: decompressobj(15 + 32) over the first member
    assert zlib.decompressobj(15 + 32).decompress(payload) == want


def test_gzip_truncated_returns_what_inflated(rplib):
    full = gzip.compress(corpus(5))
    cut = full[: len(full) // 2]
    rc, got = uncompress(rplib, abi.CODEC_GZIP, cut)
    assert rc == 0
    assert got == zlib.decompressobj(15 + 32).decompress(cut)
    assert 0 < len(got) < len(corpus(5))


def test_gzip_errors_throw(rplib):
    bad = bytearray(gzip.compress(corpus(6, 20000)))
    bad[len(bad) // 2] ^= 0xFF  # data error (or a crc mismatch in the trailer)
    crc_bad = bytearray(gzip.compress(corpus(7, 20000)))
    crc_bad[-6] ^= 1  # the CRC32 trailer
    for p in (bytes(bad), bytes(crc_bad), b"not a gzip stream at all"):
        rc, _ = uncompress(rplib, abi.CODEC_GZIP, p)
        assert rc == abi.E_CODEC


def test_gzip_overflow_reports_size(rplib):
    payload = gzip.compress(corpus(8, 50000))
    rc, need = uncompress(rplib, abi.CODEC_GZIP, payload, cap=1000)
    assert rc == abi.E_OVERFLOW and need == 50000


def test_zstd_host_fallback(rplib):
    L = zstd_lib()
    for data in (corpus(9), corpus(10, 1 << 20), b"x" * 5, bytes(np.random.default_rng(3).integers(0, 256, 70000,
                                                                                                  dtype=np.uint8))):
        frame = zstd_compress(data)
        rc, got = uncompress(rplib, abi.CODEC_ZSTD, frame)
        assert rc == 0 and got == data
        out = C.create_string_buffer(len(data) + 1)
        assert L.ZSTD_decompress(out, len(data) + 1, frame, len(frame)) == len(data)
    # frames concatenate (ZSTD_decompressStream starts the next frame)
    a, b = corpus(11, 3000), corpus(12, 4000)
    rc, got = uncompress(rplib, abi.CODEC_ZSTD, zstd_compress(a) + zstd_compress(b))
    assert rc == 0 and got == a + b


def test_zstd_errors(rplib):
    frame = zstd_compress(corpus(13, 100000))
    for p in (frame + b"\x01\x02\x03\x04garbage!", b"definitely not zstd", frame[:8] + b"\xff" * 40):
        rc, _ = uncompress(rplib, abi.CODEC_ZSTD, p)
        assert rc == abi.E_CODEC
    rc, need = uncompress(rplib, abi.CODEC_ZSTD, frame, cap=10)
    assert rc == abi.E_OVERFLOW and need == 100000


def test_zstd_short_input_is_an_empty_result(rplib):
    """Fewer bytes than a frame header: ZSTD_decompressStream consumes them and
    asks for more; the reference loop (stream_zstd.cc:160-176) then returns
    what it has, nothing."""
    assert uncompress(rplib, abi.CODEC_ZSTD, b"\x01\x02\x03") == (0, b"")
    assert uncompress(rplib, abi.CODEC_ZSTD, zstd_compress(b"abc" * 1000)[:3]) == (0, b"")


def test_empty_and_none_throw(rplib):
    assert uncompress(rplib, abi.CODEC_GZIP, b"")[0] == abi.E_CODEC
    assert uncompress(rplib, abi.CODEC_ZSTD, b"")[0] == abi.E_CODEC
    # the device codecs still need a context
    assert uncompress(rplib, abi.CODEC_LZ4, b"\x00")[0] == abi.E_INVALID


@pytest.mark.gpu
def test_host_codecs_through_context_and_batch(engine):
    """The same surface through a device context, and mixed in one
    rpgpu_uncompress_batch call with device (lz4/snappy) payloads."""
    import synth  # noqa: F401
    g = gzip.compress(corpus(14, 40000))
    z = zstd_compress(corpus(15, 40000))
    assert engine.uncompress(abi.CODEC_GZIP, g) == corpus(14, 40000)
    assert engine.uncompress(abi.CODEC_ZSTD, z) == corpus(15, 40000)
    res = engine.uncompress_batch([abi.CODEC_GZIP, abi.CODEC_ZSTD, abi.CODEC_NONE], [g, z, b"abc"])
    assert res[0] == (0, corpus(14, 40000)) and res[1] == (0, corpus(15, 40000)) and res[2][0] == abi.E_CODEC
