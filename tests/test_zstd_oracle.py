"""The oracle's zstd path (rpo_zstd_uncompress: stream_zstd::do_uncompress's
loop, compression/stream_zstd.cc:152-178, over libzstd) against librpgpu's
host fallback (rp_hostcodec.cpp, the same loop): frames from libzstd's
streaming compressor, truncations, bit flips, concatenations.  CPU only."""
from __future__ import annotations

import ctypes as C
import random

import numpy as np
import pytest

from oracle import oracle as O
from redpanda_amd import abi


def _host(L, codec, data, cap):
    src = np.frombuffer(data + b"\0" * 16, dtype=np.uint8)
    dst = np.zeros(max(cap, 1), dtype=np.uint8)
    n = C.c_size_t(0)
    rc = L.rpgpu_uncompress(None, codec, src.ctypes.data_as(C.c_void_p), len(data), dst.ctypes.data_as(C.c_void_p),
                            cap, C.byref(n))
    return rc, bytes(dst[: n.value])


def test_oracle_zstd_matches_host_fallback():
    from redpanda_amd import _lib
    from tests import compress_corpus as CC
    from tests.test_compress import _host_compress
    L = _lib.load()
    rng = random.Random(5)
    frames = []
    gens = [CC.text, CC.json_like, CC.random_bytes, CC.low_entropy]
    for k in range(12):
        data = gens[k % 4](rng.choice([0, 10, 1000, 70000, 300000]), k)
        st, f = _host_compress(_lib, abi.CODEC_ZSTD, data, rng.choice([0, 4096]))
        assert st == 0
        frames.append(f)
    cases = list(frames)
    for f in frames:
        b = bytearray(f)
        cases.append(bytes(b[: max(1, len(b) // 2)]))
        b[len(b) // 3] ^= 0x10
        cases.append(bytes(b))
        cases.append(f + f)
    for s in cases:
        cap = 1 << 22
        hrc, hout = _host(L, abi.CODEC_ZSTD, s, cap)
        orc, oout = O.uncompress(abi.CODEC_ZSTD, s, cap)
        assert (hrc == 0) == (orc == 0), (len(s), hrc, orc)
        if orc == 0:
            assert hout == oout
