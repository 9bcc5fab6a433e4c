"""Pure-Python builder of Redpanda record batches for tests.

Independent of the product's C++ generator and of the oracle: it encodes the
formats straight from the reference's layouts (SURVEY.md §8 byte layouts,
model/record_utils.cc:183-227 append_record_to_buffer, storage/
segment_appender_utils.cc:28-54 disk header) and can emit malformed records
on purpose.
"""
from __future__ import annotations

import struct

_T = []


def _table():
    if not _T:
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
            _T.append(c)
    return _T


def crc32c(data: bytes, crc: int = 0) -> int:
    t = _table()
    c = crc ^ 0xFFFFFFFF
    for b in data:
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def zigzag(v: int) -> int:
    return ((v << 1) ^ (v >> 63)) & 0xFFFFFFFFFFFFFFFF


def vint(v: int) -> bytes:
    z = zigzag(v)
    out = bytearray()
    while z >= 0x80:
        out.append((z & 0x7F) | 0x80)
        z >>= 7
    out.append(z)
    return bytes(out)


def record(i: int, key: bytes | None, value: bytes | None, headers=(), attrs: int = 0,
           ts_delta: int | None = None, off_delta: int | None = None, length: int | None = None,
           key_len: int | None = None, val_len: int | None = None, hdr_count: int | None = None) -> bytes:
    """One Kafka v2 record; *_len / hdr_count / length override the encoded
    values (malformed records)."""
    body = bytearray()
    body.append(attrs & 0xFF)
    body += vint(i if ts_delta is None else ts_delta)
    body += vint(i if off_delta is None else off_delta)
    kl = (len(key) if key is not None else -1) if key_len is None else key_len
    body += vint(kl)
    if key:
        body += key
    vl = (len(value) if value is not None else -1) if val_len is None else val_len
    body += vint(vl)
    if value:
        body += value
    body += vint(len(headers) if hdr_count is None else hdr_count)
    for hk, hv in headers:
        body += vint(len(hk)) + hk + vint(len(hv)) + hv
    return vint(len(body) if length is None else length) + bytes(body)


HDR = struct.Struct("<IiqbihiqqqhiI")  # disk header, 61 bytes
assert HDR.size == 61


def be_prefix(attrs, lod, first_ts, max_ts, pid, epoch, seq, count) -> bytes:
    return struct.pack(">hiqqqhii", attrs, lod, first_ts, max_ts, pid, epoch, seq, count)


def batch(payload: bytes, record_count: int, base_offset: int = 0, attrs: int = 0, btype: int = 1,
          first_ts: int = 1600000000000, lod: int | None = None, pid: int = -1, epoch: int = -1,
          seq: int = -1, size_bytes: int | None = None, crc: int | None = None,
          header_crc: int | None = None) -> bytes:
    """Disk-layout batch; crc/header_crc/size_bytes are computed unless given."""
    lod = record_count - 1 if lod is None else lod
    max_ts = first_ts + max(record_count - 1, 0)
    size = 61 + len(payload) if size_bytes is None else size_bytes
    if crc is None:
        crc = crc32c(payload, crc32c(be_prefix(attrs, lod, first_ts, max_ts, pid, epoch, seq, record_count)))
    crc_i = struct.unpack("<i", struct.pack("<I", crc & 0xFFFFFFFF))[0]
    fields = (size, base_offset, btype, crc_i, attrs, lod, first_ts, max_ts, pid, epoch, seq, record_count)
    body = struct.pack("<iqbihiqqqhiI", *fields[:11], record_count & 0xFFFFFFFF)
    if header_crc is None:
        header_crc = crc32c(body)
    return struct.pack("<I", header_crc) + body + payload


def simple_records(n: int, vlen: int = 40, klen: int = 8, headers: int = 2, seed: int = 1) -> bytes:
    import random
    rnd = random.Random(seed)
    alnum = b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ012345678"
    out = bytearray()
    for i in range(n):
        k = bytes(rnd.choice(alnum) for _ in range(klen))
        v = bytes(rnd.choice(alnum) for _ in range(vlen))
        hs = [(bytes(rnd.choice(alnum) for _ in range(rnd.randint(1, 10))),
               bytes(rnd.choice(alnum) for _ in range(rnd.randint(1, 10)))) for _ in range(headers)]
        out += record(i, k, v, hs)
    return bytes(out)


DISK_HDR = struct.Struct("<Iiqbihiqqqhii")   # storage/segment_appender_utils.cc:28-54
WIRE_HDR = struct.Struct(">qiibihiqqqhii")   # kafka/protocol/response_writer.h:241-276


def disk_to_wire(seg: bytes, stop_at_bad_header: bool = True) -> bytes:
    """writer_serialize_batch (kafka/protocol/response_writer.h:241-276) over
    every complete batch of a disk segment: the Kafka v2 record set the
    produce path receives (batch_length = size_bytes - 12, leader epoch 0,
    magic 2; the crc and payload are unchanged).  Stops at the first
    fallocated / incomplete batch."""
    out = bytearray()
    pos = 0
    while len(seg) - pos >= 61:
        (hcrc, size, base, typ, crc, attrs, lod, first, mx, pid, epoch, seq, rc) = DISK_HDR.unpack_from(seg, pos)
        if hcrc == 0 or size < 61 or pos + size > len(seg):
            break
        if stop_at_bad_header and crc32c(bytes(seg[pos + 4:pos + 61])) != hcrc:
            break
        out += WIRE_HDR.pack(base, size - 12, 0, 2, crc, attrs, lod, first, mx, pid, epoch, seq, rc)
        out += seg[pos + 61:pos + size]
        pos += size
    return bytes(out)


def wire_batches(rs: bytes):
    """(offset, size) of each batch of a well-formed record set."""
    pos, out = 0, []
    while len(rs) - pos >= 61:
        size = struct.unpack_from(">i", rs, pos + 8)[0] + 12
        out.append((pos, size))
        pos += size
    return out
