"""The oracle's inflate restatement (rpo_gzip_uncompress) pinned against zlib
1.2.11 (the library gzip_compressor links; Python's zlib module is the same
system library) and against the reference's own loop over it in librpgpu's
host codec (rp_hostcodec.cpp, the CPU fallback).  CPU only."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from oracle import oracle as O
from redpanda_amd import abi
from tests.gzip_corpus import clean_streams, mutated_streams, zlib_truth


def oracle_gzip(data: bytes):
    rc, out = O.uncompress(abi.CODEC_GZIP, data, cap=1)
    if rc == -2:
        # the sizing pass: retry with the full size, as the reference's second pass
        src = np.frombuffer(bytes(data) + b"\0" * 8, dtype=np.uint8)
        dst = np.zeros(1, dtype=np.uint8)
        n = C.c_size_t(0)
        O.lib().rpo_uncompress(abi.CODEC_GZIP, src.ctypes.data_as(C.c_void_p), len(data),
                               dst.ctypes.data_as(C.c_void_p), 0, C.byref(n))
        rc, out = O.uncompress(abi.CODEC_GZIP, data, cap=max(n.value, 1))
    if rc == -1:
        return None
    assert rc == 0
    return out


@pytest.mark.parametrize("kind", ["clean", "mutated"])
def test_oracle_inflate_matches_zlib(kind):
    streams = clean_streams() if kind == "clean" else mutated_streams()
    errors = partial = 0
    for i, s in enumerate(streams):
        want = zlib_truth(s)
        got = oracle_gzip(s)
        assert (got is None) == (want is None), (kind, i, len(s), want is None)
        if want is not None:
            assert got == want, (kind, i, len(s), len(got), len(want))
        errors += want is None
    if kind == "mutated":
        assert errors > 30  # the corpus exercises the reject paths


def test_oracle_inflate_every_truncation():
    # every prefix of a few small members: the partial output zlib yields
    import random
    import zlib

    from tests.gzip_corpus import gzip_member
    rng = random.Random(3)
    for strat in (zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY):
        data = bytes(rng.choice(b"abcab ") for _ in range(3000))
        for flags in (0, 30):
            s = gzip_member(data, 6, strat, flags=flags)
            for k in range(1, len(s) + 1, 3 if len(s) > 600 else 1):
                assert oracle_gzip(s[:k]) == zlib_truth(s[:k]), (strat, flags, k)
        s = gzip_member(data, 0)  # stored blocks
        for k in range(1, len(s) + 1, 7):
            assert oracle_gzip(s[:k]) == zlib_truth(s[:k]), ("stored", k)


def test_oracle_inflate_agrees_with_reference_loop():
    """The reference's loop over zlib (rp_hostcodec.cpp, no device needed)."""
    from redpanda_amd import _lib
    L = _lib.load()
    for s in clean_streams(5, 20, 30000) + mutated_streams(6, 60):
        src = np.frombuffer(s + b"\0" * 16, dtype=np.uint8)
        cap = 1 << 22
        dst = np.zeros(cap, dtype=np.uint8)
        n = C.c_size_t(0)
        rc = L.rpgpu_uncompress(None, abi.CODEC_GZIP, src.ctypes.data_as(C.c_void_p), len(s),
                                dst.ctypes.data_as(C.c_void_p), cap, C.byref(n))
        got = oracle_gzip(s)
        if rc == abi.E_CODEC:
            assert got is None
        else:
            assert rc == 0 and got == bytes(dst[: n.value])
