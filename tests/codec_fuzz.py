"""Seeded LZ4F / raw-snappy / snappy-java frame mutations (test
infrastructure).

Base frames come from the reference's codec libraries themselves (liblz4 1.9.3
/ libsnappy 1.1.8 through oracle/_ref/libcodecref.so, called the way
lz4_frame_compressor.cc:72-113 and snappy_java_compressor.cc:58-75 call
them), in every flag combination the frame formats have; the mutations are
the corruptions a segment on disk or a produce request can carry: bit flips,
byte sets, truncations, trailing bytes, inserted / deleted / duplicated
slices, zeroed runs, and edits aimed at the structural fields (LZ4F FLG / BD /
content size / header checksum / block size words and their raw bit; the
snappy length preamble and tag bytes; the snappy-java magic, version words and
big-endian chunk lengths).

Expected results are the libraries' (ref_lz4f_uncompress <-
lz4_frame_compressor.cc:115-200, ref_snappy_java <- snappy_java_compressor.cc:
76-129, ref_snappy_raw <- snappy_standard_compressor.cc:43-65).  Used by
tests/test_codec_fuzz.py (oracle vs libraries, in process) and by
tests/golden/make_codec_fuzz.py (the committed corpus the GPU test replays).
"""
from __future__ import annotations

import ctypes as C
import random

import numpy as np

LZ4 = 3
SNAPPY = 2
CAP_MIN = 1 << 20


def cap_for(data: bytes) -> int:
    """Output capacity the fixture tests use for one payload."""
    return max(len(data) * 300, CAP_MIN)


def _text(rnd: random.Random, n: int) -> bytes:
    words = [b"alpha", b"beta", b"gamma", b"{\"id\":", b"\"value\":", b"null,", b"true}", b" ", b"0123",
             b"redpanda", b"\n"]
    out = bytearray()
    while len(out) < n:
        out += rnd.choice(words)
    return bytes(out[:n])


def _payload(rnd: random.Random, n: int) -> bytes:
    k = rnd.random()
    if k < 0.45:
        return _text(rnd, n)
    if k < 0.6:
        return bytes(rnd.getrandbits(8) for _ in range(n))  # incompressible: stored blocks
    if k < 0.75:
        return bytes([rnd.getrandbits(8)]) * n  # one long run (overlapping matches)
    # mixed: runs, text and noise
    out = bytearray()
    while len(out) < n:
        r = rnd.random()
        m = rnd.randint(1, 400)
        if r < 0.4:
            out += _text(rnd, m)
        elif r < 0.7:
            out += bytes(rnd.getrandbits(8) for _ in range(m))
        else:
            out += bytes([rnd.getrandbits(8)]) * m
    return bytes(out[:n])


def _arr(b: bytes):
    a = np.frombuffer(bytes(b) + b"\0" * 16, dtype=np.uint8)
    return a, a.ctypes.data_as(C.c_void_p)


def lz4f(ref, data: bytes, linked=0, bc=0, cc=0, cs=1, bsid=4) -> bytes:
    cap = ref.ref_lz4f_bound(len(data)) + 64
    dst = np.zeros(cap, dtype=np.uint8)
    src, sp = _arr(data)
    n = ref.ref_lz4f_compress(sp, len(data), dst.ctypes.data_as(C.c_void_p), cap, linked, bc, cc, cs, bsid)
    return bytes(dst[:n])


def snappy_raw(ref, data: bytes) -> bytes:
    cap = ref.ref_snappy_bound(len(data)) + 16
    dst = np.zeros(cap, dtype=np.uint8)
    src, sp = _arr(data)
    n = ref.ref_snappy_compress(sp, len(data), dst.ctypes.data_as(C.c_void_p), cap)
    return bytes(dst[:n])


def snappy_java(ref, data: bytes, chunk=4096, min_version=1, version=1) -> bytes:
    o = bytearray(b"\x82SNAPPY\0" + version.to_bytes(4, "little") + min_version.to_bytes(4, "little", signed=True))
    for i in range(0, len(data), chunk):
        c = snappy_raw(ref, data[i:i + chunk])
        o += len(c).to_bytes(4, "big") + c
    return bytes(o)


def base_frames(ref, rnd: random.Random, n: int, max_in: int = 6000):
    """n (codec, kind, frame) from the libraries, every flag combination."""
    out = []
    for i in range(n):
        size = rnd.choice([0, 1, 5, 17, 64, 300, 1000, 4000, max_in, rnd.randint(1, max_in)])
        data = _payload(rnd, size)
        k = i % 10
        if k < 6:
            kw = dict(linked=rnd.random() < 0.35, bc=rnd.random() < 0.3, cc=rnd.random() < 0.4,
                      cs=rnd.random() < 0.6, bsid=rnd.choice([4, 4, 4, 5]))
            f = lz4f(ref, data, **{a: int(b) for a, b in kw.items()})
            if size > 300 and rnd.random() < 0.3:  # several 64 KiB blocks need > 64 KiB: make small ones instead
                f = lz4f(ref, data + data[: rnd.randint(0, size)], **{a: int(b) for a, b in kw.items()})
            out.append((LZ4, "lz4f", f))
        elif k < 8:
            out.append((SNAPPY, "raw", snappy_raw(ref, data)))
        else:
            out.append((SNAPPY, "java", snappy_java(ref, data, chunk=rnd.choice([64, 512, 4096]),
                                                    min_version=rnd.choice([1, 1, 1, 0, 2]),
                                                    version=rnd.choice([1, 1, 0x01000000]))))
    return out


def _lz4f_fields(f: bytes):
    """Byte positions of an LZ4F frame's structural fields (as far as they
    parse): FLG, BD, header checksum, block size words."""
    pos = {"flg": 4, "bd": 5}
    if len(f) < 7:
        return pos, []
    flg = f[4]
    h = 6 + (8 if flg & 0x08 else 0) + (4 if flg & 0x01 else 0)
    pos["hc"] = h
    pos["csize"] = 6 if flg & 0x08 else None
    words = []
    p = h + 1
    while p + 4 <= len(f) and len(words) < 64:
        w = int.from_bytes(f[p:p + 4], "little")
        words.append(p)
        if w == 0:
            break
        p += 4 + (w & 0x7FFFFFFF) + (4 if flg & 0x10 else 0)
    return pos, words


def mutate(rnd: random.Random, codec: int, kind: str, f: bytes) -> bytes:
    """One seeded corruption of frame f."""
    b = bytearray(f)
    n = len(b)
    op = rnd.randrange(14)
    if n == 0:
        return bytes(rnd.getrandbits(8) for _ in range(rnd.randint(1, 8)))
    if op == 0:  # 1..4 bit flips anywhere
        for _ in range(rnd.randint(1, 4)):
            i = rnd.randrange(n)
            b[i] ^= 1 << rnd.randrange(8)
    elif op == 1:  # a byte set to 0x00 / 0xFF / random
        b[rnd.randrange(n)] = rnd.choice([0, 0xFF, rnd.getrandbits(8)])
    elif op == 2:  # truncation
        b = b[: rnd.randrange(n)]
    elif op == 3:  # trailing bytes
        b += bytes(rnd.getrandbits(8) for _ in range(rnd.randint(1, 16)))
    elif op == 4:  # delete a slice
        i = rnd.randrange(n)
        del b[i:i + rnd.randint(1, 32)]
    elif op == 5:  # insert random bytes
        i = rnd.randrange(n + 1)
        b[i:i] = bytes(rnd.getrandbits(8) for _ in range(rnd.randint(1, 8)))
    elif op == 6:  # duplicate a slice
        i = rnd.randrange(n)
        j = min(n, i + rnd.randint(1, 64))
        b[j:j] = b[i:j]
    elif op == 7:  # zero a run
        i = rnd.randrange(n)
        for k in range(i, min(n, i + rnd.randint(1, 24))):
            b[k] = 0
    elif op == 8:  # swap two bytes
        i, j = rnd.randrange(n), rnd.randrange(n)
        b[i], b[j] = b[j], b[i]
    elif codec == LZ4:
        pos, words = _lz4f_fields(f)
        if op == 9 and words:  # a block size word: raw bit, size +- small, huge
            p = rnd.choice(words)
            w = int.from_bytes(b[p:p + 4], "little")
            w = rnd.choice([w ^ 0x80000000, (w + rnd.randint(-3, 3)) & 0xFFFFFFFF, 0x7FFFFFFF, w & 0x80000000,
                            (w & 0x80000000) | rnd.randint(1, 70000)])
            b[p:p + 4] = w.to_bytes(4, "little")
        elif op == 10:  # FLG / BD bits (header checksum left stale or recomputed)
            k = rnd.choice(["flg", "bd"])
            b[pos[k]] ^= 1 << rnd.randrange(8)
            if "hc" in pos and rnd.random() < 0.6 and pos["hc"] < n:
                import xxhash
                hc = pos["hc"]
                b[hc] = (xxhash.xxh32(bytes(b[4:hc]), seed=0).intdigest() >> 8) & 0xFF
        elif op == 11 and pos.get("csize") is not None and pos["csize"] + 8 <= n:  # content size field
            p = pos["csize"]
            v = int.from_bytes(b[p:p + 8], "little")
            v = rnd.choice([0, v + 1, max(v - 1, 0), v * 2, 1 << 40])
            b[p:p + 8] = v.to_bytes(8, "little")
            import xxhash
            hc = pos["hc"]
            if hc < n:
                b[hc] = (xxhash.xxh32(bytes(b[4:hc]), seed=0).intdigest() >> 8) & 0xFF
        elif op == 12 and words and len(words) > 1:  # a block's body: flip inside it
            p = rnd.choice(words[:-1])
            w = int.from_bytes(b[p:p + 4], "little") & 0x7FFFFFFF
            if w:
                i = p + 4 + rnd.randrange(w)
                if i < n:
                    b[i] ^= 1 << rnd.randrange(8)
        else:  # token byte near the first block's start
            if words:
                i = words[0] + 4 + rnd.randrange(4)
                if i < n:
                    b[i] = rnd.getrandbits(8)
    elif kind == "raw":
        if op == 9:  # the length preamble
            b[0] = rnd.getrandbits(8)
        elif op == 10:  # a tag byte early in the stream
            i = min(n - 1, rnd.randrange(1, 6))
            b[i] = rnd.getrandbits(8)
        elif op == 11:  # preamble longer / shorter
            if rnd.random() < 0.5:
                b[0:0] = bytes([0x80 | rnd.getrandbits(7)])
            else:
                del b[0]
        else:  # a copy offset byte
            i = rnd.randrange(n)
            b[i] = rnd.choice([0, 1, 0xFF])
    else:  # snappy-java
        if op == 9 and n >= 16:  # magic / version / min_version
            i = rnd.randrange(16)
            b[i] ^= 1 << rnd.randrange(8)
        elif op == 10 and n >= 20:  # the first chunk's BE length
            v = int.from_bytes(b[16:20], "big")
            v = rnd.choice([v + 1, max(v - 1, 0), 0, 0x80000000, 0x7FFFFFFF, v + 1000])
            b[16:20] = (v & 0xFFFFFFFF).to_bytes(4, "big")
        elif op == 11 and n >= 16:  # min_version below 1 / version words
            b[12:16] = rnd.choice([0, -1, 2, 0x7FFFFFFF]).to_bytes(4, "little", signed=True)
        else:  # inside the first chunk body
            if n > 21:
                i = 20 + rnd.randrange(n - 20)
                b[i] ^= 1 << rnd.randrange(8)
    return bytes(b)


def ref_uncompress(ref, codec: int, kind: str, data: bytes, cap: int):
    """(rc, bytes) from the libraries: rc 0 ok, -1 the reference throws, -2
    capacity too small."""
    fn = ref.ref_lz4f_uncompress if codec == LZ4 else ref.ref_snappy_java
    src, sp = _arr(data)
    dst = np.zeros(max(cap, 1), dtype=np.uint8)
    out = C.c_size_t(0)
    rc = fn(sp, len(data), dst.ctypes.data_as(C.c_void_p), cap, C.byref(out))
    return rc, bytes(dst[: out.value]) if rc == 0 else b""


def corpus(ref, seed: int, n_base: int, per_base: int, max_in: int = 6000):
    """[(codec, kind, frame)]: the base frames and per_base mutations of each."""
    rnd = random.Random(seed)
    out = []
    for codec, kind, f in base_frames(ref, rnd, n_base, max_in):
        out.append((codec, kind, f))
        for _ in range(per_base):
            out.append((codec, kind, mutate(rnd, codec, kind, f)))
    return out
