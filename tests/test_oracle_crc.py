"""Oracle CRC32C / XXH32 / vint pinned by published vectors."""
import os
import random

import numpy as np


def test_crc32c_check_value(oracle):
    # CRC-32C check value ("123456789")
    assert oracle.crc32c(b"123456789") == 0xE3069283


def test_crc32c_rfc3720_vectors(oracle):
    # RFC 3720 appendix B.4
    assert oracle.crc32c(bytes(32)) == 0x8A9136AA
    assert oracle.crc32c(b"\xff" * 32) == 0x62A8AB43
    assert oracle.crc32c(bytes(range(32))) == 0x46DD794E
    assert oracle.crc32c(bytes(range(31, -1, -1))) == 0x113FDB5C
    iscsi = bytes.fromhex("01c00000000000000000000000000000"
                          "14000000000004000000001400000018"
                          "28000000000000000200000000000000")
    assert oracle.crc32c(iscsi) == 0xD9963A56


def test_crc32c_extend_is_incremental(oracle):
    """crc::crc32c::extend over fragments == one call (iobuf fragments)."""
    rnd = random.Random(7)
    data = bytes(rnd.getrandbits(8) for _ in range(5000))
    c = 0
    for i in range(0, len(data), 333):
        c = oracle.crc32c(data[i:i + 333], c)
    assert c == oracle.crc32c(data)


def test_crc32c_hw_matches_table(oracle):
    rnd = random.Random(3)
    for n in (0, 1, 7, 8, 63, 4096 * 3 + 5, 100000):
        d = bytes(rnd.getrandbits(8) for _ in range(n))
        for seed in (0, 0xDEADBEEF):
            assert oracle.crc32c_hw(d, seed) == oracle.crc32c(d, seed)


def test_xxh32_vectors(oracle):
    # published XXH32 test values
    assert oracle.xxh32(b"", 0) == 0x02CC5D05
    assert oracle.xxh32(b"a", 0) == 0x550D7456
    assert oracle.xxh32(b"abc", 0) == 0x32D153FF
    assert oracle.xxh32(b"Nobody inspects the spammish repetition", 0) == 0xE2293B2F


def test_vint_quirks(oracle):
    """utils/vint.h:82-98 behaviours named in SURVEY §8(a) a11."""
    assert oracle.vint_deserialize(b"") == (0, 0)
    assert oracle.vint_deserialize(b"\xff" * 12) == (-(1 << 63), 10)   # 10-byte cap
    assert oracle.vint_deserialize(b"\x80\x80") == (0, 2)               # truncated: partial value
    for v in (0, 1, -1, 63, -64, 64, 1 << 31, -(1 << 62), (1 << 63) - 1, -(1 << 63)):
        enc = oracle.vint_serialize(v)
        assert oracle.vint_deserialize(enc) == (v, len(enc))
    # utils/tests/vint_test.cc sweep: +-1e8 step 1e5
    for v in range(-100_000_000, 100_000_001, 100_000):
        enc = oracle.vint_serialize(v)
        assert oracle.vint_deserialize(enc + b"\x01") == (v, len(enc))
