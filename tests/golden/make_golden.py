#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/.

Run in the build container (where /root/reference exists); the outputs are
data only (inputs + expected outputs) and are what the CPU tests check the
oracle against.  Sources of truth:

* segment fixtures: bytes built by tests/batchgen.py, expected header fields,
  CRC verdicts and record fields produced by the reference's own Python
  segment reader, tools/metadata_viewer/storage.py (+ reader.py), imported
  from /root/reference with a pure-Python `crc32c` module standing in for the
  pinned crc32c==2.2.post0 wheel (absent here).  Where the Python tool and the
  C++ broker disagree (null lengths, varint cap, EOF), the case
  is marked `python_ref: false` and only the C++-derived expectation is kept;
* codec fixtures: frames produced by liblz4 1.9.3 / libsnappy 1.1.8 and
  mutations of them, expected outputs from the same libraries driven the way
  the reference's wrappers drive them (oracle/codec_ref.c).
"""
from __future__ import annotations

import hashlib
import io
import json
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import batchgen as bg  # noqa: E402

REF_TOOL = "/root/reference/tools/metadata_viewer"


def load_reference_reader():
    shim = types.ModuleType("crc32c")
    shim.crc32c = lambda data, value=0: bg.crc32c(bytes(data), value)
    sys.modules["crc32c"] = shim
    sys.path.insert(0, REF_TOOL)
    import storage  # the reference's tools/metadata_viewer/storage.py
    return storage


def ref_parse_segment(storage, seg: bytes):
    """Iterate the segment with the reference reader; returns per-batch
    verdicts until the first CorruptBatchError / end."""
    out = []
    f = io.BytesIO(seg)
    idx = 0
    while True:
        pos = f.tell()
        try:
            b = storage.Batch.from_stream(f, idx)
        except storage.CorruptBatchError as e:
            h = e.batch.header
            out.append({"file_pos": pos, "valid": False, "header": list(h)})
            break
        except AssertionError:
            out.append({"file_pos": pos, "truncated": True})
            break
        if b is None:
            break
        recs = []
        for r in b:
            recs.append({"length": r.length, "attrs": r.attrs, "ts_delta": r.timestamp_delta,
                         "offset_delta": r.offset_delta, "key_len": len(r.key), "val_len": len(r.value),
                         "hdr_count": len(r.headers)})
        out.append({"file_pos": pos, "valid": True, "header": list(b.header), "records": recs})
        idx += 1
    return out


def segment_cases():
    """(name, segment bytes, python_ref usable, note)"""
    C = []
    p = bg.simple_records(5)
    ok = bg.batch(p, 5, base_offset=0)
    C.append(("ok_single", ok, True, "one valid batch"))
    ten = b"".join(bg.batch(bg.simple_records(3, seed=i), 3, base_offset=3 * i) for i in range(10))
    C.append(("ten_valid", ten, True, "10 valid batches"))
    # log_replayer_test.cc:118-183 behaviours
    bad_crc = bg.batch(p, 5, crc=10)
    C.append(("crc_is_10", bad_crc, True, "crc=10 -> not recovered"))
    b = bytearray(ok)
    b[27:35] = (1700000000000).to_bytes(8, "little")  # first_timestamp changed, header_crc restamped
    hb = bytes(b)
    hb = bg.crc32c(hb[4:61]).to_bytes(4, "little") + hb[4:]
    C.append(("first_ts_changed", hb, True, "changed first_timestamp -> crc mismatch"))
    last_bad = b"".join(bg.batch(bg.simple_records(3, seed=i), 3, base_offset=3 * i,
                                 crc=(10 if i == 9 else None)) for i in range(10))
    C.append(("last_of_ten_corrupt", last_bad, True, "recovered up to batch 9"))
    C.append(("garbage", bytes(range(256)) * 4, False, "garbage file -> not recovered"))
    # header corruption, zero header, short tail
    hc = bytearray(ten)
    hc[61 * 0 + len(bg.batch(bg.simple_records(3, seed=0), 3)) + 9] ^= 0x10
    C.append(("header_bitflip_batch1", bytes(hc), False, "header_crc mismatch stops the chain"))
    C.append(("zero_header_tail", ok + bytes(200), True, "fallocated zeros -> benign end"))
    C.append(("short_tail", ok + ok[:40], False, "fewer than 61 bytes after the last batch"))
    C.append(("truncated_records", ok + ok[:-7], False, "last batch payload truncated"))
    # codec values 5..7
    C.append(("codec_bits_5", bg.batch(p, 5, attrs=5), True, "compression() throws for 5..7"))
    # record-level quirks (C++ semantics; Python tool differs)
    nulls = bg.record(0, None, None, []) + bg.record(1, b"k", None, [(b"h", b"v")])
    C.append(("null_key_value", bg.batch(nulls, 2), False, "key/value length -1 -> nothing read"))
    neg_hc = bg.record(0, b"k", b"v", [], hdr_count=-1)
    C.append(("negative_header_count", bg.batch(neg_hc, 1), False, "headers.reserve(-1) throws"))
    big = bytes([0xFF] * 9 + [0x01])  # 10-byte varint as ts delta
    r10 = bytes([(1 + 1 + 10 + 1 + 1 + 1 + 1 + 1) * 2]) + b"\x00" + big + b"\x00" + b"\x02k" + b"\x02v" + b"\x00"
    C.append(("ten_byte_varint", bg.batch(r10, 1), False, "10-byte varint accepted"))
    overrun = bg.record(0, b"k", b"v", []) + bg.record(1, b"kk", None, [], key_len=50)
    C.append(("key_overrun_last_record", bg.batch(overrun, 2), False,
              "key length past the end: copy is silent, async walk accepts"))
    trailing = bg.record(0, b"k", b"v", []) + b"\x00\x00\x00"
    C.append(("trailing_bytes", bg.batch(trailing, 1), False, "sync for_each_record rejects trailing bytes"))
    attr_eof = bg.record(0, b"k", b"v", [])
    C.append(("record_count_too_big", bg.batch(attr_eof, 3), False, "attr read at EOF throws"))
    zero_rc = bg.batch(b"", 0)
    C.append(("empty_batch", zero_rc, True, "record_count 0, empty payload"))
    neg_copy = bg.record(0, b"", b"", [], key_len=(1 << 31) + 5)
    C.append(("negative_int_copy", bg.batch(neg_copy, 1), False, "(int)len < 0 -> bad_alloc"))
    # headers the discovery prefilter rejects although read_header_impl
    # accepts them (storage/parser.cc:139-176 validates neither type nor
    # size nor offsets): the chain must run through them
    def chain(mid: bytes) -> bytes:
        return (bg.batch(bg.simple_records(3, seed=40), 3, base_offset=0) + mid +
                bg.batch(bg.simple_records(2, seed=41), 2, base_offset=100))
    C.append(("type_zero_mid_chain", chain(bg.batch(bg.simple_records(2, seed=42), 2, base_offset=3, btype=0)),
              True, "record_batch_type 0 chains"))
    C.append(("type_99_mid_chain", chain(bg.batch(bg.simple_records(2, seed=43), 2, base_offset=3, btype=99)),
              True, "record_batch_type 99 chains"))
    C.append(("negative_base_offset_mid_chain",
              chain(bg.batch(bg.simple_records(2, seed=44), 2, base_offset=-5)), True,
              "negative base_offset chains"))
    C.append(("codec_6_mid_chain", chain(bg.batch(bg.simple_records(2, seed=45), 2, base_offset=3, attrs=6)),
              True, "codec bits 6: crc ok, compression() throws, chain continues"))
    C.append(("negative_record_count_mid_chain",
              chain(bg.batch(bg.simple_records(2, seed=46), -1, base_offset=3, lod=1)), False,
              "record_count -1 chains; no record is walked"))
    small = bg.batch(b"", 0, base_offset=3, size_bytes=40)
    C.append(("size_40_valid_header_crc", bg.batch(bg.simple_records(3, seed=47), 3) + small + bytes(100), False,
              "size_bytes 40 (< 61) with a valid header_crc: size-61 unsigned -> not enough bytes"))
    return C


def codec_cases(ref):
    import ctypes as C
    import numpy as np
    import random
    rnd = random.Random(0xC0DEC)
    out = []

    def comp_lz4(data, **kw):
        cap = ref.ref_lz4f_bound(len(data))
        dst = np.zeros(cap, dtype=np.uint8)
        src = np.frombuffer(data + b"\0", dtype=np.uint8)
        n = ref.ref_lz4f_compress(src.ctypes.data_as(C.c_void_p), len(data), dst.ctypes.data_as(C.c_void_p), cap,
                                  kw.get("linked", 0), kw.get("bc", 0), kw.get("cc", 0), kw.get("cs", 1),
                                  kw.get("bsid", 4))
        return bytes(dst[:n])

    def comp_snappy(data):
        cap = ref.ref_snappy_bound(len(data))
        dst = np.zeros(cap, dtype=np.uint8)
        src = np.frombuffer(data + b"\0", dtype=np.uint8)
        n = ref.ref_snappy_compress(src.ctypes.data_as(C.c_void_p), len(data), dst.ctypes.data_as(C.c_void_p), cap)
        return bytes(dst[:n])

    def snappy_java(data, chunk=4096, min_version=1, version=1):
        o = bytearray(b"\x82SNAPPY\0" + version.to_bytes(4, "little") + min_version.to_bytes(4, "little", signed=True))
        for i in range(0, len(data), chunk):
            c = comp_snappy(data[i:i + chunk])
            o += len(c).to_bytes(4, "big") + c
        return bytes(o)

    text = bytes(rnd.choice(b"abcdefghij0123456789 ") for _ in range(70000))
    rnd_bytes = bytes(rnd.getrandbits(8) for _ in range(5000))
    rep = b'{"user":7,"event":"click"}' * 3000
    lz = comp_lz4(text)
    out += [
        ("lz4_indep_cs", 3, lz),
        ("lz4_linked", 3, comp_lz4(rep, linked=1, cs=0)),
        ("lz4_block_checksum", 3, comp_lz4(text[:20000], bc=1)),
        ("lz4_content_checksum", 3, comp_lz4(rep, cc=1)),
        ("lz4_random_stored", 3, comp_lz4(rnd_bytes, cs=0)),
        ("lz4_256k_blocks", 3, comp_lz4(text * 5, bsid=5)),
        ("lz4_truncated_after_block", 3, lz[:len(lz) - 4]),
        ("lz4_truncated_mid", 3, lz[: len(lz) // 2]),
        ("lz4_trailing_garbage", 3, lz + b"\x01\x02"),
        ("lz4_two_frames", 3, lz + lz),
        ("lz4_bad_header_checksum", 3, lz[:6] + bytes([lz[6] ^ 1]) + lz[7:]),
        ("lz4_bad_magic", 3, b"\x05" + lz[1:]),
        ("lz4_skippable", 3, (0x184D2A5A).to_bytes(4, "little") + (3).to_bytes(4, "little") + b"abc"),
        ("lz4_empty_input", 3, b""),
        ("snappy_java", 2, snappy_java(text)),
        ("snappy_java_le_version_big", 2, snappy_java(rep, version=0x01000000)),
        ("snappy_java_min_version_0", 2, snappy_java(rep, min_version=0)),
        ("snappy_raw", 2, comp_snappy(text[:30000])),
        ("snappy_raw_empty_frame", 2, b"\x00garbage-after-zero-length"),
        ("snappy_raw_bad_offset", 2, b"\x0a\x08abc\x0d\x09\x00"),
        ("snappy_java_truncated_chunk", 2, snappy_java(text)[:-10]),
    ]
    # deterministic single-byte mutations of a few frames
    for name, codec, base in [("lz4_mut", 3, comp_lz4(text[:3000], bc=1, cc=1)), ("snappy_mut", 2, snappy_java(rep[:5000]))]:
        for k in range(6):
            b = bytearray(base)
            i = rnd.randrange(len(b))
            b[i] ^= 1 << rnd.randrange(8)
            out.append((f"{name}_{k}", codec, bytes(b)))
    return out


def main():
    storage = load_reference_reader()
    from oracle import oracle as O
    O.build()
    ref = O.ref()
    assert ref is not None, "liblz4/libsnappy harness not buildable"
    seg_dir = os.path.join(HERE, "segments")
    codec_dir = os.path.join(HERE, "codecs")
    os.makedirs(seg_dir, exist_ok=True)
    os.makedirs(codec_dir, exist_ok=True)
    manifest = {"segments": [], "codecs": []}
    for name, seg, use_py, note in segment_cases():
        with open(os.path.join(seg_dir, name + ".bin"), "wb") as f:
            f.write(seg)
        ent = {"name": name, "note": note, "bytes": len(seg), "python_ref": use_py}
        if use_py:
            ent["reference_reader"] = ref_parse_segment(storage, seg)
        manifest["segments"].append(ent)
    import ctypes as C
    import numpy as np
    for name, codec, data in codec_cases(ref):
        with open(os.path.join(codec_dir, name + ".bin"), "wb") as f:
            f.write(data)
        cap = max(len(data) * 300, 1 << 20)
        src = np.frombuffer(data + b"\0" * 8, dtype=np.uint8)
        dst = np.zeros(cap, dtype=np.uint8)
        n = C.c_size_t(0)
        if len(data) == 0:
            rc = -1  # compressor::uncompress throws on an empty buffer
        elif codec == 3:
            rc = ref.ref_lz4f_uncompress(src.ctypes.data_as(C.c_void_p), len(data), dst.ctypes.data_as(C.c_void_p), cap, C.byref(n))
        else:
            rc = ref.ref_snappy_java(src.ctypes.data_as(C.c_void_p), len(data), dst.ctypes.data_as(C.c_void_p), cap, C.byref(n))
        out = bytes(dst[: n.value]) if rc == 0 else b""
        manifest["codecs"].append({"name": name, "codec": codec, "rc": int(rc), "out_len": len(out),
                                   "out_sha256": hashlib.sha256(out).hexdigest(),
                                   "library": "liblz4 1.9.3" if codec == 3 else "libsnappy 1.1.8"})
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"wrote {len(manifest['segments'])} segment and {len(manifest['codecs'])} codec fixtures")


if __name__ == "__main__":
    main()
