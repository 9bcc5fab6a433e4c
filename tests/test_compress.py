"""Write side, compression: compressor::compress for
lz4 and snappy (compression/compression.cc:17-33) as
storage::internal::compress_batch calls it (storage/parser_utils.cc:97-111).

Oracle: rp_oracle.c's restatement of liblz4 1.9.3 LZ4_compress_generic (as
lz4_frame_compressor.cc:72-113 drives it through LZ4F) and libsnappy 1.1.8
CompressFragment (as snappy_java_compressor.cc:58-75 drives RawCompress).
Pinned two ways: against the libraries themselves through the reference's
wrapper loops (oracle/_ref, when buildable) and against golden sha256 vectors
of those outputs (tests/golden/compress_vectors.json, made by
golden/make_compress_golden.py).  The GPU (rpgpu_compress_batch) is compared
with the oracle byte for byte, and its frames decode back (on the device and
through the reference's libraries).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import compress_corpus as CC
from redpanda_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "compress_vectors.json")))
NAMES = {3: "lz4", 2: "snappy"}


@pytest.fixture(scope="module")
def corpus():
    return CC.cases()


def test_oracle_matches_golden_vectors(oracle, corpus):
    from oracle import oracle as O
    n = 0
    for name, data in corpus:
        for codec in (3, 2):
            for frag in (CC.FRAGS if codec == 2 else (0,)):
                r = O.compress(codec, data, frag)
                want = GOLD[f"{NAMES[codec]}/{name}/{frag}"]
                assert [len(r), hashlib.sha256(r).hexdigest()] == want, (codec, name, frag)
                n += 1
    assert n == len(GOLD)


def test_oracle_matches_reference_libraries(oracle):
    """Fresh random payloads (not in the golden set) against liblz4 /
    libsnappy through the reference's loops; lz4 frames are the same
    whatever the iobuf fragmentation."""
    from oracle import oracle as O
    if O.ref() is None:
        pytest.skip("oracle/_ref harness not buildable here; the golden vectors pin the oracle")
    rng = np.random.default_rng(0xC0DE)
    makers = [CC.text, CC.json_like, CC.random_bytes, CC.low_entropy, CC.mostly_random]
    for i in range(40):
        n = int(rng.choice([rng.integers(0, 300), rng.integers(300, 70000), rng.integers(70000, 400000)]))
        data = makers[i % len(makers)](n, 1000 + i)
        for codec in (3, 2):
            for frag in (0, int(rng.integers(1, 200000))):
                assert O.compress(codec, data, frag) == O.ref_compress(codec, data, frag), (i, codec, n, frag)


def test_oracle_round_trip(oracle, corpus):
    """What the oracle compresses, the oracle's decoders (pinned on the read
    side) give back."""
    from oracle import oracle as O
    for name, data in corpus:
        for codec in (3, 2):
            frame = O.compress(codec, data, 1000 if codec == 2 else 0)
            st, got = O.uncompress(codec, frame)
            assert st == 0 and got == data, (name, codec)


def test_compress_bound(rplib, corpus):
    from oracle import oracle as O
    L = rplib.load()
    for name, data in corpus:
        for codec in (3, 2):
            for frag in (0, 1000):
                b = L.rpgpu_compress_bound(codec, len(data), frag)
                assert b >= len(O.compress(codec, data, frag)), (name, codec, frag)
    assert L.rpgpu_compress_bound(abi.CODEC_NONE, 100, 0) == 0


@pytest.mark.gpu
def test_gpu_compress_matches_oracle(engine, corpus):
    """rpgpu_compress_batch == the oracle byte for byte over the corpus, lz4
    and snappy-java at several fragment sizes, in one batch."""
    from oracle import oracle as O
    codecs, pays, frags = [], [], []
    for name, data in corpus:
        for codec in (3, 2):
            # odd fragment sizes (1001, 4097) put fragment starts at every
            # byte alignment of the caller's buffer
            for frag in ((0, 1000, 1001, 4097, 100_000) if codec == 2 else (0,)):
                codecs.append(codec)
                pays.append(data)
                frags.append(frag)
    res = engine.compress_batch(codecs, pays, frags)
    for (st, got), codec, data, frag in zip(res, codecs, pays, frags):
        assert st == 0
        assert got == O.compress(codec, data, frag), (codec, len(data), frag)


@pytest.mark.gpu
def test_gpu_compress_round_trip_and_statuses(engine):
    """Frames decode back on the device (rpgpu_uncompress_batch); none throws,
    gzip / zstd go to the host in the same call; a too-small capacity
    reports the size needed."""
    data = [CC.json_like(1 << 20, 11), CC.text(200_000, 12), CC.random_bytes(70000, 13), b"abc" * 7]
    codecs = [3, 2, 3, 2]
    res = engine.compress_batch(codecs, data)
    assert all(st == 0 for st, _ in res)
    back = engine.uncompress_batch(codecs, [f for _, f in res], caps=[len(d) + 64 for d in data])
    assert [b for _, b in back] == data
    st = engine.compress_batch([abi.CODEC_NONE, abi.CODEC_GZIP, abi.CODEC_ZSTD], [b"x" * 10] * 3)
    assert [s for s, _ in st] == [abi.E_CODEC, abi.OK, abi.OK]
    assert engine.uncompress_batch([abi.CODEC_GZIP, abi.CODEC_ZSTD], [st[1][1], st[2][1]]) == [(0, b"x" * 10)] * 2
    full = engine.compress_batch([3], [data[0]])[0][1]
    st, need = engine.compress_batch([3], [data[0]], caps=[100])[0]
    assert st == abi.E_OVERFLOW and need == len(full)


@pytest.mark.gpu
def test_gpu_compress_many_blocks(engine):
    """Several hundred blocks in one call (the scratch slots, the pack's
    fragment walk): 48 payloads of 64 KiB .. 2 MiB."""
    from oracle import oracle as O
    rng = np.random.default_rng(5)
    makers = [CC.text, CC.json_like, CC.mostly_random, CC.low_entropy]
    pays = [makers[i % 4](int(rng.integers(65536, 2 << 20)), 100 + i) for i in range(48)]
    codecs = [3 if i % 2 else 2 for i in range(48)]
    frags = [0 if i % 3 else 131072 for i in range(48)]
    res = engine.compress_batch(codecs, pays, frags)
    for (st, got), codec, data, frag in zip(res, codecs, pays, frags):
        assert st == 0 and got == O.compress(codec, data, frag)


def _host_compress(rplib, codec, data, frag=0, cap=None):
    """rpgpu_compress_batch with a NULL context (gzip / zstd are host work)."""
    import ctypes as C
    L = rplib.load()
    src = np.frombuffer(bytes(data), dtype=np.uint8) if data else np.zeros(1, np.uint8)
    cap = cap if cap is not None else L.rpgpu_compress_bound(codec, len(data), frag)
    out = np.zeros(max(cap, 1), np.uint8)
    ci, ip = (C.c_int * 1)(codec), (C.c_void_p * 1)(src.ctypes.data)
    il, fr = (C.c_size_t * 1)(len(data)), (C.c_size_t * 1)(frag)
    op, oc, ol, st = (C.c_void_p * 1)(out.ctypes.data), (C.c_size_t * 1)(cap), (C.c_size_t * 1)(), (C.c_int * 1)()
    assert L.rpgpu_compress_batch(None, 1, ci, ip, il, fr, op, oc, ol, st) == 0
    return int(st[0]), (out[: ol[0]].tobytes() if st[0] == 0 else int(ol[0]))


def test_gzip_compress_host_fallback(rplib, corpus):
    """gzip_compressor::compress (gzip_compressor.cc:126-161): deflateInit2(
    Z_DEFAULT_COMPRESSION, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY), one
    deflate per fragment, Z_FINISH — byte for byte what Python's zlib
    (an independent driver of the same library, same parameters) gives."""
    import zlib
    for name, data in corpus:
        for frag in (0, 1000):
            st, got = _host_compress(rplib, abi.CODEC_GZIP, data, frag)
            c = zlib.compressobj(-1, zlib.DEFLATED, 31, 8, 0)
            want = b"".join(c.compress(data[f:f + (frag or len(data) or 1)])
                            for f in range(0, len(data), frag or len(data) or 1)) + c.flush()
            assert st == 0 and got == want, (name, frag)
            assert zlib.decompress(got, 31) == data


def test_zstd_compress_host_fallback(rplib, corpus):
    """stream_zstd::do_compress (stream_zstd.cc:84-104): the frame carries the
    content size and decodes back through libzstd and the host uncompress
    path; per-fragment flushes make distinct (valid) frames."""
    import test_hostcodec as H
    Z = H.zstd_lib()
    import ctypes as C
    Z.ZSTD_getFrameContentSize.restype = C.c_ulonglong
    Z.ZSTD_getFrameContentSize.argtypes = [C.c_void_p, C.c_size_t]
    for name, data in corpus:
        for frag in (0, 1000):
            st, frame = _host_compress(rplib, abi.CODEC_ZSTD, data, frag)
            assert st == 0, name
            assert Z.ZSTD_getFrameContentSize(frame, len(frame)) == len(data)
            rc, back = H.uncompress(rplib, abi.CODEC_ZSTD, frame, cap=len(data) + 1)
            assert rc == 0 and back == data, (name, frag)


def test_host_compress_overflow_and_none(rplib):
    data = CC.text(50000, 3)
    st, full = _host_compress(rplib, abi.CODEC_GZIP, data)
    st2, need = _host_compress(rplib, abi.CODEC_GZIP, data, cap=10)
    assert st == 0 and st2 == abi.E_OVERFLOW and need == len(full)
    assert _host_compress(rplib, abi.CODEC_NONE, data, cap=100)[0] == abi.E_CODEC
    # device codecs need a context
    assert _host_compress(rplib, abi.CODEC_LZ4, data)[0] == abi.E_INVALID
