"""GPU parity of the LZ4 block walk (k_lzf_walk + k_lzf_tail, round 5) on
hand-built LZ4F frames: every case the lane walk hands to the reference loop
or rejects on its own, through the job pipeline (not the lane engine of
rpgpu_uncompress), against the oracle's restatement of LZ4_decompress_generic
(oracle/rp_oracle.c, liblz4 1.9.3 semantics) field by field.

Cases per frame (one 64 KiB independent block each unless noted):
  * literal runs of 0..14, 15..254 and >= 270 bytes (one and several
    length-extension bytes: the walk's straight-line step vs its hand-off),
    runs of 200..270 bytes (the lane window is restaged mid-sequence);
  * matches of 4..18, 19..273 and >= 274 bytes, offsets 1..15 (overlapping
    copies) up to the whole block behind;
  * offset 0 mid-block, an offset reaching before the block, a block cut
    short, a match ending inside the last 5 / starting inside the last 12
    output bytes, literals not ending the stream exactly (the reference
    loop's end rules, which the walk leaves to k_lzf_tail);
  * linked-block frames (their matches reaching into the previous block)
    and records compressed by the oracle's LZ4F writer.
"""
import os
import random
import sys

import numpy as np
import pytest

from redpanda_amd import abi

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import batchgen as bg  # noqa: E402
from test_gpu_parity import assert_same, run_both  # noqa: E402

pytestmark = pytest.mark.gpu
DFLAGS = abi.JOB_CRC | abi.JOB_PARSE | abi.JOB_DECODE
LZ4 = 3


def ext(v: int) -> bytes:
    out = bytearray()
    while v >= 255:
        out.append(255)
        v -= 255
    out.append(v)
    return bytes(out)


def seq(lit: bytes, off: int = 0, ml: int = 0) -> bytes:
    """One LZ4 sequence: literals, then a match (ml = 0: the last sequence)."""
    ll = len(lit)
    m = ml - 4 if ml else 0
    out = bytearray([(min(ll, 15) << 4) | (min(m, 15) if ml else 0)])
    if ll >= 15:
        out += ext(ll - 15)
    out += lit
    if ml:
        out += off.to_bytes(2, "little")
        if m >= 15:
            out += ext(m - 15)
    return bytes(out)


def frame(blocks, linked=False, raw=(), bcs=False, content=None) -> bytes:
    """LZ4F frame, 64 KiB blocks; blocks whose index is in `raw` are stored
    (uncompressed, size word bit 31); bcs = a block checksum after every
    block; content = the decoded bytes, whose XXH32 then follows the end mark
    (the content-checksum flag)."""
    import xxhash
    flg = 0x40 | (0 if linked else 0x20) | (0x10 if bcs else 0) | (0x04 if content is not None else 0)
    bd = 0x40
    hc = (xxhash.xxh32(bytes([flg, bd]), seed=0).intdigest() >> 8) & 0xFF
    out = bytearray(b"\x04\x22\x4d\x18" + bytes([flg, bd, hc]))
    for i, b in enumerate(blocks):
        out += (len(b) | (0x80000000 if i in raw else 0)).to_bytes(4, "little") + b
        if bcs:
            out += xxhash.xxh32(b, seed=0).intdigest().to_bytes(4, "little")
    out += b"\x00\x00\x00\x00"
    if content is not None:
        out += xxhash.xxh32(content, seed=0).intdigest().to_bytes(4, "little")
    return bytes(out)


def text(rnd, n):
    words = [b"alpha", b"beta", b"gamma", b"delta", b"{\"id\":", b"\"value\":", b"null,", b"true}", b" "]
    out = bytearray()
    while len(out) < n:
        out += rnd.choice(words)
    return bytes(out[:n])


def valid_block(rnd, kind):
    """A block that decodes (LZ4 end rules kept) and its output."""
    out = bytearray()
    parts = []
    limit = 60000
    while len(out) < limit - 4000:
        r = rnd.random()
        if kind == "long_lits" and r < 0.3:
            ll = rnd.randint(270, 900)
        elif kind == "restage" and r < 0.4:
            ll = rnd.randint(200, 270)
        elif r < 0.5:
            ll = rnd.randint(0, 14)
        else:
            ll = rnd.randint(15, 120)
        lit = bytes(rnd.getrandbits(8) for _ in range(ll)) if kind != "text" else text(rnd, ll)
        out += lit
        if not out:
            continue
        if kind == "long_match" and r < 0.3:
            ml = rnd.randint(274, 3000)
        elif r < 0.6:
            ml = rnd.randint(4, 18)
        else:
            ml = rnd.randint(19, 273)
        if rnd.random() < 0.25:
            off = rnd.randint(1, min(15, len(out)))
        else:
            off = rnd.randint(1, min(len(out), 65535))
        parts.append(seq(lit, off, ml))
        for _ in range(ml):
            out.append(out[-off])
    last = bytes(rnd.getrandbits(8) for _ in range(rnd.randint(5, 40)))
    parts.append(seq(last))
    out += last
    return b"".join(parts), bytes(out)


def bad_blocks(rnd):
    """Blocks the reference rejects (or accepts by its own end rules)."""
    cases = []
    base, _ = valid_block(rnd, "mixed")
    # offset 0 in the middle
    cases.append(seq(b"abcdefgh", 4, 8) + seq(b"ij", 0, 6) + seq(b"tail-bytes-12"))
    # offset before the block start
    cases.append(seq(b"abcd", 9, 8) + seq(b"tail-bytes-12"))
    # cut short at many places
    for cut in (1, 2, 7, 33, len(base) // 2, len(base) - 3, len(base) - 1):
        cases.append(base[:cut])
    # a match ending inside the last 5 output bytes / literals after it too short
    cases.append(seq(b"x" * 20, 10, 20) + seq(b"abc"))
    cases.append(seq(b"y" * 30, 1, 40) + seq(b""))
    # the last literals do not end the stream exactly (trailing garbage)
    cases.append(seq(b"z" * 16, 3, 9) + seq(b"end-of-block!") + b"\x00\x11")
    # a length extension running past the block
    cases.append(bytes([0xF0]) + b"\xff" * 6)
    cases.append(seq(b"q" * 8, 2, 8) + bytes([0x0F, 0x02, 0x00]) + b"\xff" * 5)
    # random byte flips in a valid block (the walk's verdicts vs the reference's)
    for _ in range(24):
        b = bytearray(base)
        for _ in range(rnd.randint(1, 4)):
            b[rnd.randrange(len(b))] = rnd.getrandbits(8)
        cases.append(bytes(b))
    return cases


def segment(payloads) -> np.ndarray:
    out = bytearray()
    off = 0
    for p in payloads:
        n = 3
        out += bg.batch(p, n, base_offset=off, attrs=LZ4)
        off += n
    return np.frombuffer(bytes(out), dtype=np.uint8).copy()


@pytest.mark.parametrize("seed", [1, 2])
def test_lz4_walk_edge_blocks(engine, oracle, seed):
    rnd = random.Random(seed)
    frames = []
    for kind in ("mixed", "text", "long_lits", "restage", "long_match"):
        for _ in range(4):
            blk, _ = valid_block(rnd, kind)
            frames.append(frame([blk]))
    for blk in bad_blocks(rnd):
        frames.append(frame([blk]))
    # two-block frames: independent, and linked (matches into block 0)
    for _ in range(4):
        b0, o0 = valid_block(rnd, "text")
        b1, _ = valid_block(rnd, "mixed")
        frames.append(frame([b0, b1]))
        lk = seq(b"L" * 10, 50000, 300) + seq(text(rnd, 40), len(o0) + 5, 64) + seq(b"tail-bytes-12")
        frames.append(frame([b0, lk], linked=True))
    rnd.shuffle(frames)
    segs = [segment(frames[i::2]) for i in range(2)]
    got, ref = run_both(engine, oracle, segs, flags=DFLAGS)
    f = ref.batches["flags"]
    assert np.any(f & abi.F_CODEC_OK) and not np.all(f & abi.F_CODEC_OK)
    assert_same(got, ref, DFLAGS)


def test_lz4_walk_compressed_records(engine, oracle):
    """Records with incompressible runs between repeated text, compressed by
    the oracle's LZ4F writer (lz4_frame_compressor.cc:72-113 restated)."""
    rnd = random.Random(7)
    payloads = []
    for b in range(40):
        recs = []
        for i in range(rnd.randint(20, 200)):
            r = rnd.random()
            if r < 0.3:
                v = bytes(rnd.getrandbits(8) for _ in range(rnd.randint(280, 700)))
            elif r < 0.5:
                v = bytes([rnd.getrandbits(8)]) * rnd.randint(300, 3000)
            else:
                v = text(rnd, rnd.randint(10, 400))
            recs.append(bg.record(i, b"k%d" % i, v))
        raw = b"".join(recs)
        payloads.append((oracle.compress(LZ4, raw), len(recs)))
    out = bytearray()
    off = 0
    for p, n in payloads:
        out += bg.batch(p, n, base_offset=off, attrs=LZ4)
        off += n
    seg = np.frombuffer(bytes(out), dtype=np.uint8).copy()
    got, ref = run_both(engine, oracle, [seg], flags=DFLAGS)
    f = ref.batches["flags"]
    assert np.all(f & abi.F_CODEC_OK) and np.all(f & abi.F_PARSE_OK)
    assert_same(got, ref, DFLAGS)


def raw_block_frames(rnd):
    """Frames mixing stored (raw) blocks with compressed ones: independent raw
    blocks without a block checksum go to k_raw_copy (BlockItem.fast =
    kLzfRaw, its streaming crc combined into the frame's), the compressed ones
    to k_lzf_walk; a raw block under a block checksum, and every block of a
    linked frame, stay on the lane walk / exec."""
    def rawb(n):
        return text(rnd, n) if rnd.random() < 0.5 else bytes(rnd.getrandbits(8) for _ in range(n))
    frames = []
    for _ in range(3):
        b0, o0 = valid_block(rnd, "mixed")
        b2, o2 = valid_block(rnd, "text")
        r1, r3 = rawb(65536), rawb(rnd.randint(1, 65536))
        # a raw block between / after compressed ones, with and without a content checksum
        frames.append(frame([b0, r1, b2], raw=(1,)))
        frames.append(frame([b0, r1, b2, r3], raw=(1, 3), content=o0 + r1 + o2 + r3))
        # raw blocks first and last
        frames.append(frame([r1, b0, r3], raw=(0, 2)))
        frames.append(frame([r1, b2, r3], raw=(0, 2), content=r1 + o2 + r3))
        # every block raw, with a content checksum; a damaged content checksum
        frames.append(frame([r1, r3], raw=(0, 1), content=r1 + r3))
        bad = bytearray(frame([r3, b0], raw=(0,), content=r3 + o0))
        bad[-1] ^= 0x40
        frames.append(bytes(bad))
        # raw blocks under a block checksum (the lane walk's), one damaged
        frames.append(frame([b0, r1, r3], raw=(1, 2), bcs=True))
        frames.append(frame([r3, b2], raw=(0,), bcs=True, content=r3 + o2))
        bad = bytearray(frame([b0, r3], raw=(1,), bcs=True))
        bad[-6] ^= 0x01  # the raw block's checksum
        frames.append(bytes(bad))
        # a linked frame whose compressed block copies from the raw block before it
        lk = seq(b"R" * 7, len(r1) - 10, 200) + seq(text(rnd, 30), 40000, 70) + seq(b"tail-bytes-12")
        frames.append(frame([r1, lk], linked=True, raw=(0,)))
        frames.append(frame([b0, r1, lk], linked=True, raw=(1,)))
    return frames


@pytest.mark.parametrize("seed", [3, 4])
def test_lz4_walk_raw_blocks(engine, oracle, seed):
    """stored blocks beside walked ones, content and block
    checksums, raw blocks in linked frames."""
    rnd = random.Random(seed)
    frames = raw_block_frames(rnd)
    rnd.shuffle(frames)
    segs = [segment(frames[i::2]) for i in range(2)]
    got, ref = run_both(engine, oracle, segs, flags=DFLAGS)
    f = ref.batches["flags"]
    assert np.sum((f & abi.F_CODEC_OK) != 0) >= len(frames) - 8 and not np.all(f & abi.F_CODEC_OK)
    assert_same(got, ref, DFLAGS)
