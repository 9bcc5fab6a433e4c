"""Kafka v2 wire layout: the oracle's restatement of
kafka::batch_reader + kafka_batch_adapter::adapt (kafka/protocol/
batch_reader.cc:50-156, kafka_batch_adapter.cc:32-188), pinned by

* the cases of the reference's own kafka/protocol/tests/batch_reader_test.cc
  (random batches serialised by writer_serialize_batch; last_offset; short
  header -> corrupt_message; magic / crc / last_offset_delta corrupted as
  that test does, by decrementing the native int32 at the field offset);
* equivalence with the disk layout: a disk segment re-serialised for the
  wire must give the same CRC verdicts, records and checkpoint, and the
  adapted header's internal_header_only_crc must equal the disk header_crc
  (an independent check of the BE field decoding).
"""
import struct

import numpy as np
import pytest

from redpanda_amd import abi
from tests import batchgen as bg
import synth  # noqa: E402  (test/bench data generator, not the product)

FLAGS = abi.JOB_CRC | abi.JOB_PARSE
MAG_OFFSET = 8 + 4 + 4          # batch_reader_test.cc:76-78
CRC_OFFSET = MAG_OFFSET + 1     # :79-80
LOD_OFFSET = CRC_OFFSET + 4 + 2  # :81-83


def gen(rplib, nbytes, idx, **kw):
    a = np.zeros(nbytes, dtype=np.uint8)
    synth.gen_segment(a, idx, **kw)
    return a


def run(oracle, rs: bytes, layout=abi.LAYOUT_WIRE, flags=FLAGS):
    arr = np.frombuffer(rs, dtype=np.uint8)
    return oracle.run_job(arr, np.array([0, len(rs)], np.uint64), flags, layout=layout)


def corrupt_i32(rs: bytes, off: int) -> bytes:
    """corrupt_offset<int32_t>(..., [](int32_t& t) { --t; }) (native LE)."""
    b = bytearray(rs)
    v = struct.unpack_from("<i", b, off)[0]
    struct.pack_into("<i", b, off, (v - 1 + 2**31) % 2**32 - 2**31)
    return bytes(b)


@pytest.fixture(scope="module")
def record_set(rplib):
    seg = gen(rplib, 400_000, 0, seed=42, batch_bytes=0, min_batch=300, max_batch=20_000)
    rs = bg.disk_to_wire(seg.tobytes())
    assert len(bg.wire_batches(rs)) >= 40
    return seg.tobytes(), rs


def test_last_offset_and_consume_all(oracle, record_set):
    """batch_reader_last_offset / consumer_records_consume_batch."""
    _, rs = record_set
    r = run(oracle, rs)
    f = r.batches["flags"]
    assert np.all(f & abi.F_WIRE_V2) and np.all(f & abi.F_CRC_OK) and np.all(f & abi.F_PARSE_OK)
    sm = r.summaries[0]
    assert sm["first_bad"] == len(r.batches) and sm["terminal_errc"] == abi.ERRC_END_OF_STREAM
    last = r.batches[-1]
    assert sm["ckpt_last_offset"] == int(last["base_offset"]) + int(last["last_offset_delta"])
    assert sm["bytes_consumed"] == len(rs) == sm["ckpt_truncate_pos"]
    assert np.all(r.batches["type"] == 1)  # raft_data


def test_short_header(oracle, record_set):
    """batch_reader_last_offset_short_header: trim_back(size - 61 + 3)."""
    _, rs = record_set
    short = rs[: len(rs) - (len(rs) - 61 + 3)]  # 58 bytes: less than one header
    r = run(oracle, short)
    assert len(r.batches) == 0
    assert r.summaries[0]["terminal_errc"] == abi.ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES


@pytest.mark.parametrize("field,off", [("magic", MAG_OFFSET), ("crc", CRC_OFFSET), ("lod", LOD_OFFSET)])
def test_corrupt_first_batch(oracle, record_set, field, off):
    """consumer_records_consume_batch_fail_{magic,crc} and
    batch_reader_record_batch_reader_impl_fail_{crc,lod}."""
    _, rs = record_set
    r = run(oracle, corrupt_i32(rs, off))
    b0 = r.batches[0]
    if field == "magic":
        assert not b0["flags"] & abi.F_WIRE_V2
    else:
        assert b0["flags"] & abi.F_WIRE_V2
    assert not b0["flags"] & abi.F_CRC_OK        # !valid_crc (or never computed)
    assert not b0["flags"] & abi.F_PARSED        # adapt() returned before the parse
    assert r.summaries[0]["first_bad"] == 0 and r.summaries[0]["has_checkpoint"] == 0
    assert r.summaries[0]["bytes_consumed"] == 0
    # the chain itself is structural: every batch is still found
    assert len(r.batches) == len(bg.wire_batches(rs))


def test_malformed_lengths(oracle, record_set):
    _, rs = record_set
    batches = bg.wire_batches(rs)
    # batch 3 cut short: recorded incomplete, chain ends at eof
    p3, s3 = batches[3]
    r = run(oracle, rs[: p3 + s3 - 5])
    assert len(r.batches) == 4 and not r.batches[3]["flags"] & abi.F_COMPLETE
    sm = r.summaries[0]
    assert sm["first_bad"] == 3 and sm["terminal_eof"] == 1
    assert sm["terminal_errc"] == abi.ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES
    # batch_length too small to hold a header: adapt() would throw
    b = bytearray(rs)
    struct.pack_into(">i", b, p3 + 8, 20)
    r = run(oracle, bytes(b))
    assert len(r.batches) == 3 and r.summaries[0]["terminal_pos"] == p3
    assert r.summaries[0]["terminal_errc"] == abi.ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES


def fix_crc(b: bytearray, pos: int, size: int):
    struct.pack_into(">I", b, pos + 17, bg.crc32c(bytes(b[pos + 21:pos + size])))


def test_codec_bits_and_parse_failure_stop_the_read(oracle, record_set):
    _, rs = record_set
    batches = bg.wire_batches(rs)
    # codec bits 5..7 with a matching crc: compressed() throws inside adapt
    # (model/record.h:283-300), so the read stops there
    p2, s2 = batches[2]
    b = bytearray(rs)
    b[p2 + 22] = (b[p2 + 22] & ~7) | 6
    fix_crc(b, p2, s2)
    r = run(oracle, bytes(b))
    f2 = r.batches[2]["flags"]
    assert f2 & abi.F_CRC_OK and f2 & abi.F_CODEC_INVALID and not f2 & abi.F_PARSED
    assert r.summaries[0]["first_bad"] == 2 and r.summaries[0]["bytes_consumed"] == p2
    # one record more than the payload holds, crc matching: the sync
    # for_each_record throws (model/record.h:616-627)
    p4, s4 = batches[4]
    b = bytearray(rs)
    rc = struct.unpack_from(">i", b, p4 + 57)[0]
    struct.pack_into(">i", b, p4 + 57, rc + 1)
    fix_crc(b, p4, s4)
    r = run(oracle, bytes(b))
    f4 = r.batches[4]["flags"]
    assert f4 & abi.F_CRC_OK and f4 & abi.F_PARSED and not f4 & abi.F_PARSE_OK
    assert r.summaries[0]["first_bad"] == 4


def test_wire_equals_disk(oracle, rplib):
    """The same batches as a disk segment and as a record set: identical
    verdicts, records and checkpoint; adapted header_crc == disk header_crc."""
    for seed, kw in [(7, dict(corrupt_payload_ppm=150_000)), (8, dict(value_bytes=60)), (9, {})]:
        seg = gen(rplib, 300_000, 1, seed=seed, batch_bytes=0, min_batch=200, max_batch=30_000, **kw).tobytes()
        rs = bg.disk_to_wire(seg)
        d = run(oracle, seg, layout=abi.LAYOUT_DISK)
        w = run(oracle, rs)
        n = len(bg.wire_batches(rs))
        db, wb = d.batches[:n], w.batches
        assert len(wb) == n
        for f in ("base_offset", "first_timestamp", "max_timestamp", "producer_id", "size_bytes", "record_count",
                  "last_offset_delta", "base_sequence", "crc", "crc_computed", "attrs", "producer_epoch"):
            np.testing.assert_array_equal(wb[f], db[f], err_msg=f)
        np.testing.assert_array_equal(wb["header_crc_computed"], db["header_crc"])
        # adapt() parses only batches whose crc matched; elsewhere the disk
        # path (which walks every complete batch) has the parse bits on top
        ok = (db["flags"] & abi.F_CRC_OK) != 0
        parse_bits = np.uint32(abi.F_PARSED | abi.F_PARSE_ASYNC_OK | abi.F_PARSE_OK | abi.F_INDEX_WRITTEN)
        want = np.where(ok, db["flags"], db["flags"] & ~parse_bits)
        np.testing.assert_array_equal(wb["flags"] & ~np.uint32(abi.F_WIRE_V2), want)
        np.testing.assert_array_equal(wb["records_parsed"][ok], db["records_parsed"][ok])
        np.testing.assert_array_equal(wb["index_base"], db["index_base"])
        for i in np.nonzero(ok)[0]:
            lo, k = int(db["index_base"][i]), int(db["records_parsed"][i])
            for f in ("rec_pos", "ts_delta", "length", "offset_delta", "key_len", "val_len", "hdr_count", "end_pos"):
                np.testing.assert_array_equal(w.records[f][lo:lo + k], d.records[f][lo:lo + k], err_msg=f)
        assert w.summaries[0]["first_bad"] == d.summaries[0]["first_bad"]
        assert w.summaries[0]["ckpt_last_offset"] == d.summaries[0]["ckpt_last_offset"]
