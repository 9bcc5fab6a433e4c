"""Deterministic payloads for the compressor parity tests (test_compress.py)
and their golden vectors (golden/make_compress_golden.py): text-like,
JSON-like, random, low-entropy, long runs, and sizes around every threshold
of the two compressors (LZ4: 13-byte minimum, 64 KiB blocks, the raw-block
decision; snappy: 15-byte margin, table sizes 256..16384, 64 KiB blocks)."""
import numpy as np


def _words(rng, n):
    return [bytes(rng.integers(97, 123, rng.integers(2, 10), dtype=np.uint8)) for _ in range(n)]


def text(n, seed):
    rng = np.random.default_rng(seed)
    w = _words(rng, 400)
    return b" ".join(w[i] for i in rng.integers(0, len(w), n // 4 + 1))[:n]


def json_like(n, seed):
    rng = np.random.default_rng(seed)
    keys = [b'"id"', b'"user"', b'"ts"', b'"value"', b'"tags"', b'"ok"']
    parts = []
    size = 0
    while size < n:
        rec = b"{" + b",".join(k + b":" + str(int(rng.integers(0, 10 ** int(rng.integers(1, 9))))).encode() for k in keys) + b"}\n"
        parts.append(rec)
        size += len(rec)
    return b"".join(parts)[:n]


def random_bytes(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def low_entropy(n, seed):
    return np.random.default_rng(seed).integers(0, 3, n, dtype=np.uint8).tobytes()


def mostly_random(n, seed):
    """random with sparse repeats: compressible by a hair (the raw-block edge)"""
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, n, dtype=np.uint8)
    for _ in range(max(1, n // 2000)):
        if n > 64:
            p, q = rng.integers(0, n - 32, 2)
            a[q:q + 16] = a[p:p + 16]
    return a.tobytes()


def cases():
    """[(name, bytes)]"""
    out = [("empty", b""), ("one", b"a"), ("run13", b"x" * 13), ("run100k", b"x" * 100_000),
           ("abc15", b"abc" * 5)]
    for n in (12, 13, 14, 15, 16, 17, 255, 256, 257, 4095, 4096, 16383, 16384, 16385, 65535, 65536, 65537):
        out.append((f"text{n}", text(n, n)))
    out += [("text1m", text(1 << 20, 1)), ("json300k", json_like(300_000, 2)), ("json70k", json_like(70_000, 9)),
            ("rand200k", random_bytes(200_000, 3)), ("rand64k", random_bytes(65536, 4)),
            ("low150k", low_entropy(150_000, 5)), ("mostly_rand131k", mostly_random(131072, 6)),
            ("mostly_rand65k", mostly_random(65536, 7)), ("rand_tail", text(65536, 8) + random_bytes(3000, 8))]
    return out


FRAGS = (0, 1000, 65536, 100_000)
