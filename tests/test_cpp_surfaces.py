"""The C++ drop-in surfaces (include/rpgpu_redpanda.h) driven through
tests/cpp/surfaces_main.cpp.

CPU tests: crc::crc32c, model::record_batch_attributes and the model:: CRC
helpers, walking generated and golden segments on the host; compared with
the oracle's per-batch verdicts.

GPU tests: storage::continuous_batch_parser replays the device verdicts into
a scripted batch_consumer; every event (accept_batch_start, consume/skip
batch start, consume_records, consume_batch_end) and every consume() result
must equal RefParser below, a restatement of continuous_batch_parser
(storage/parser.cc:96-254) over the raw segment bytes.  log_replayer and
compressor::uncompress are compared with the oracle.
"""
import os
import struct
import subprocess

import numpy as np
import pytest

from redpanda_amd import abi
from tests import batchgen as bg
import synth  # noqa: E402  (test/bench data generator, not the product)

HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")
M64 = (1 << 64) - 1


@pytest.fixture(scope="session")
def driver(rplib):
    from redpanda_amd import build as B
    return B.build_surfaces_test()


def run(driver, *args):
    r = subprocess.run([driver] + [str(a) for a in args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout.splitlines()


def gen(rplib, nbytes, idx, **kw):
    a = np.zeros(nbytes, dtype=np.uint8)
    synth.gen_segment(a, idx, **kw)
    return a


def segment_cases(rplib):
    """(name, bytes): clean, corrupted, truncated mid-payload, truncated
    mid-header, fallocated tail, header corruption, golden segments."""
    v = gen(rplib, 600_000, 0, seed=31, batch_bytes=0, min_batch=200, max_batch=60_000)
    c = gen(rplib, 600_000, 1, seed=32, batch_bytes=0, min_batch=200, max_batch=60_000, corrupt_payload_ppm=200_000)
    h = gen(rplib, 600_000, 2, seed=33, batch_bytes=0, min_batch=200, max_batch=60_000, corrupt_header_ppm=60_000)
    cases = [("clean", v.tobytes()), ("payload_corrupt", c.tobytes()), ("header_corrupt", h.tobytes())]
    # cut inside the 5th batch's payload / header, and a zero (fallocated) tail
    pos, ends = 0, []
    raw = v.tobytes()
    while len(ends) < 6:
        size = struct.unpack_from("<i", raw, pos + 4)[0]
        ends.append((pos, size))
        pos += size
    p5, s5 = ends[5]
    cases.append(("cut_payload", raw[: p5 + 61 + (s5 - 61) // 2]))
    cases.append(("cut_header", raw[: p5 + 30]))
    cases.append(("zero_tail", raw[:p5] + bytes(4096)))
    cases.append(("empty", b""))
    import json
    man = json.load(open(os.path.join(G, "manifest.json")))
    for e in man["segments"]:
        cases.append(("golden_" + e["name"], open(os.path.join(G, "segments", e["name"] + ".bin"), "rb").read()))
    return cases


def write(tmp_path, name, data):
    p = tmp_path / (name + ".seg")
    p.write_bytes(data)
    return str(p)


# ---------------------------------------------------------------------------
# CPU: model:: surfaces
# ---------------------------------------------------------------------------

def test_model_surfaces_match_oracle(driver, rplib, oracle, tmp_path):
    for name, data in segment_cases(rplib):
        lines = run(driver, "cpu", write(tmp_path, name, data))
        assert lines[0] == "SELF 0", (name, lines[0])
        got = [tuple(int(x) for x in ln.split()[1:]) for ln in lines[1:]]
        arr = np.frombuffer(data, dtype=np.uint8)
        ref = oracle.run_job(arr, np.array([0, len(data)], np.uint64), abi.JOB_CRC)
        want = [(int(b["file_pos"]), int(b["size_bytes"]), int(b["base_offset"]), 1,
                 int(bool(b["flags"] & abi.F_CRC_OK)), int(b["attrs"]))
                for b in ref.batches if b["flags"] & abi.F_COMPLETE]
        assert got == want, name


# ---------------------------------------------------------------------------
# GPU: storage::continuous_batch_parser, log_replayer, compressor
# ---------------------------------------------------------------------------

class RefParser:
    """continuous_batch_parser (storage/parser.cc:96-254) over raw bytes, with
    the same scripted consumer as surfaces_main.cpp.  Input-stream model:
    read_exactly(n) returns min(n, remaining) bytes and sets eof when short."""

    def __init__(self, seg, m, r, s, e, crc):
        self.seg, self.m, self.r, self.s, self.e, self.crc = seg, m, r, s, e, crc
        self.pos = 0
        self.eof = False
        self.header = None
        self.bytes = 0
        self.phys = 0
        self.err = 0
        self.k = 0
        self.stopped = False
        self.ev = []

    def read_exactly(self, n):
        take = min(n, len(self.seg) - self.pos)
        b = self.seg[self.pos: self.pos + take]
        self.pos += take
        if take < n:
            self.eof = True
        return b

    def read_header(self):  # read_header_impl, parser.cc:139-176
        b = self.read_exactly(61)
        if not b:
            return abi.ERRC_END_OF_STREAM
        if len(b) != 61:
            return abi.ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES
        hcrc, size, base = struct.unpack_from("<Iiq", b, 0)
        if hcrc == 0:
            return abi.ERRC_FALLOCATED_FILE_READ_ZERO_BYTES_FOR_HEADER
        if self.crc(b[4:61]) != hcrc:
            return abi.ERRC_HEADER_ONLY_CRC_MISSMATCH
        return (size, base, struct.unpack_from("<i", b, 57)[0])

    def accept(self, h):
        self.ev.append(f"ASK {self.k} {h[1]}")
        if self.k == self.s and not self.stopped:
            self.stopped = True
            return "stop"
        if self.m > 0 and self.k % self.m == self.r:
            return "skip"
        return "accept"

    def consume_header(self):  # parser.cc:96-132
        while True:
            if self.header is None:
                h = self.read_header()
                if isinstance(h, int):
                    return ("err", h)
                self.header = h
            size, base, rc = self.header
            ret = self.accept(self.header)
            if ret == "stop":
                return ("stop", None)
            if ret == "accept":
                self.ev.append(f"START {self.k} {base} {self.phys} {size & M64} {rc}")
                self.phys = (self.phys + size) & M64
                return ("no", None)
            self.ev.append(f"SKIP {self.k} {base} {self.phys} {size & M64}")
            self.k += 1
            self.phys = (self.phys + size) & M64
            rem = (size - 61) & M64
            if len(self.read_exactly(rem)) != rem:
                return ("err", abi.ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES)
            self.bytes = (self.bytes + size) & M64
            self.header = None

    def consume_one(self):  # parser.cc:178-213
        st = self.consume_header()
        if st[0] != "no":
            return st
        size = self.header[0]
        rem = (size - 61) & M64
        b = self.read_exactly(rem)
        if len(b) != rem:
            out = ("err", abi.ERRC_INPUT_STREAM_NOT_ENOUGH_BYTES)
        else:
            self.ev.append(f"RECORDS {self.k} {len(b)} {self.crc(b)}")
            stop = self.k == self.e
            self.ev.append(f"END {self.k} {int(stop)}")
            self.k += 1
            out = ("stop" if stop else "no", None)
        self.bytes = (self.bytes + size) & M64
        self.header = None
        return out

    def consume(self):  # parser.cc:218-254
        if self.err:
            self.ev.append(f"RESULT err {self.err}")
            return
        while True:
            s = self.consume_one()
            if self.eof:
                break
            if s[0] == "err":
                self.err = s[1]
                break
            if s[0] == "stop":
                break
        benign = (abi.ERRC_NONE, abi.ERRC_END_OF_STREAM, abi.ERRC_FALLOCATED_FILE_READ_ZERO_BYTES_FOR_HEADER)
        if self.bytes or self.err in benign:
            self.ev.append(f"RESULT ok {self.bytes}")
        else:
            self.ev.append(f"RESULT err {self.err}")


SCRIPTS = [(0, 0, -1, -1), (3, 1, -1, -1), (0, 0, 5, -1), (2, 0, 4, 7), (1, 0, -1, -1), (4, 3, 0, 2)]


@pytest.mark.gpu
def test_continuous_batch_parser_replay(driver, rplib, oracle, engine, tmp_path):
    for name, data in segment_cases(rplib):
        path = write(tmp_path, name, data)
        for sc in SCRIPTS:
            got = run(driver, "parse", path, *sc)
            ref = RefParser(data, *sc, crc=oracle.crc32c)
            for _ in range(3):
                ref.consume()
            assert got == ref.ev, (name, sc)


@pytest.mark.gpu
def test_continuous_batch_parser_stream(driver, rplib, oracle, engine, tmp_path):
    """The parser over an input stream (storage/parser.h:94-136 takes an
    ss::input_stream; log_replayer.cc:95-114 reads the file from position 0)
    read ahead in windows from 64 bytes (smaller than any batch: the window
    doubles) to larger than the segment: the events are the reference's."""
    for name, data in segment_cases(rplib):
        path = write(tmp_path, name, data)
        golden = name.startswith("golden_")
        for w in ((64,) if golden else (64, 1000, 20000, 1 << 20)):
            for sc in SCRIPTS[: 1 if golden else 3]:
                got = run(driver, "parse_stream", path, *sc, w)
                ref = RefParser(data, *sc, crc=oracle.crc32c)
                for _ in range(3):
                    ref.consume()
                assert got == ref.ev, (name, sc, w)


@pytest.mark.gpu
def test_log_replayer_checkpoint(driver, rplib, oracle, engine, tmp_path):
    for name, data in segment_cases(rplib):
        (line,) = run(driver, "recover", write(tmp_path, name, data))
        arr = np.frombuffer(data, dtype=np.uint8)
        sm = oracle.run_job(arr, np.array([0, len(data)], np.uint64), abi.JOB_CRC).summaries[0]
        want = f"CKPT 1 {int(sm['ckpt_last_offset'])} {int(sm['ckpt_truncate_pos'])}" if sm["has_checkpoint"] \
            else "CKPT 0"
        assert line == want, name


def test_xxh64_matches_xxhash(driver, tmp_path):
    """rpgpu::xxh64 (the index checksum, hashing/xx.h incremental_xxhash64 with
    seed 0) against the xxhash package over every tail-length path."""
    import xxhash
    rng = np.random.default_rng(7)
    for n in list(range(0, 70)) + [1000, 4099]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        (line,) = run(driver, "xxh64", write(tmp_path, f"x{n}", b))
        assert int(line) == xxhash.xxh64_intdigest(b), n


def serialize_index(st, ro, rt, ps) -> bytes:
    """index_state::checksum_and_serialize (storage/index_state.cc:189-236) with
    the checksum of checksum_state (:27-48): XXH64 (seed 0) of the LE fields."""
    import struct
    import xxhash
    n = len(ro)
    body = struct.pack("<Iqqqq", 0, int(st["base_offset"]), int(st["max_offset"]), int(st["base_timestamp"]),
                       int(st["max_timestamp"]))
    body += struct.pack("<I", n) + np.asarray(ro, "<u4").tobytes() + np.asarray(rt, "<u4").tobytes() \
        + np.asarray(ps, "<u8").tobytes()
    return struct.pack("<bIQ", 3, 8 + len(body), xxhash.xxh64_intdigest(body)) + body


@pytest.mark.gpu
def test_log_replayer_segment_index(driver, rplib, oracle, engine, tmp_path):
    """log_replayer::recover(.., index_state&) rebuilds the sparse index like
    checksumming_consumer -> segment_index::maybe_track; checked against the
    oracle's restatement over the oracle's own job results."""
    for name, data in segment_cases(rplib):
        arr = np.frombuffer(data, dtype=np.uint8)
        job = oracle.run_job(arr, np.array([0, len(data)], np.uint64), abi.JOB_CRC)
        base = int(job.batches["base_offset"][0]) if len(job.batches) else 0
        (st, ro, rt, ps), = oracle.segment_index(job.batches, job.summaries, [base])
        qs = [base - 1, base, base + 7, int(st["max_offset"]) + 5]
        lines = run(driver, "index", write(tmp_path, name, data), base, *qs)
        if int(st["assert_batch"]) >= 0:
            # a tracked batch below the index base: the reference vasserts
            # (storage/index_state.cc:55-58); the C++ surface throws there
            assert lines == ["VASSERT"], name
            continue
        sm = job.summaries[0]
        want = [f"CKPT 1 {int(sm['ckpt_last_offset'])} {int(sm['ckpt_truncate_pos'])}" if sm["has_checkpoint"]
                else "CKPT 0"]
        want.append(f"STATE {base} {int(st['max_offset'])} {int(st['base_timestamp'])} {int(st['max_timestamp'])} "
                    f"{len(ro)}")
        want += [f"E {int(a)} {int(b)} {int(c)}" for a, b, c in zip(ro, rt, ps)]
        want.append("SER " + serialize_index(st, ro, rt, ps).hex())
        want.append("HYDRATE 1 1")
        # index_state::hydrate_from_buffer's iobuf_parser throws on a short read
        want.append("HYDRATE_SHORT out_of_range out_of_range")
        for q in qs:
            if q < base or len(ro) == 0:
                want.append("NEAR none")
                continue
            i = int(np.searchsorted(ro, np.uint32(q - base), side="right")) - 1
            want.append("NEAR none" if i < 0 else f"NEAR {base + int(ro[i])} {int(ps[i])}")
        assert lines == want, name


@pytest.mark.gpu
def test_compressor_uncompress(driver, oracle, engine, tmp_path):
    import json
    man = json.load(open(os.path.join(G, "manifest.json")))
    args = []
    for ent in man["codecs"]:
        args += [ent["codec"], os.path.join(G, "codecs", ent["name"] + ".bin"), str(tmp_path / (ent["name"] + ".out"))]
    lines = run(driver, "uncompress", *args)  # one process (one HIP context) for every fixture
    assert len(lines) == len(man["codecs"])
    for ent, line in zip(man["codecs"], lines):
        src = os.path.join(G, "codecs", ent["name"] + ".bin")
        out = str(tmp_path / (ent["name"] + ".out"))
        data = open(src, "rb").read()
        rc, want = oracle.uncompress(ent["codec"], data, max(len(data) * 300, 1 << 20))
        if rc == 0:
            assert line == f"U ok {len(want)}", ent["name"]
            assert open(out, "rb").read() == want, ent["name"]
        else:
            assert line == "U runtime_error", ent["name"]
    # compression.cc:34-53: empty input and codec none throw runtime_error;
    # gzip / zstd run the reference's loops on the host (CPU fallback):
    # malformed streams throw runtime_error, good ones decode
    empty = str(tmp_path / "empty.bin")
    open(empty, "wb").close()
    one = str(tmp_path / "one.bin")
    open(one, "wb").write(b"\x01\x02\x03")
    assert run(driver, "uncompress", abi.CODEC_GZIP, empty, out) == ["U runtime_error"]
    assert run(driver, "uncompress", abi.CODEC_NONE, one, out) == ["U runtime_error"]
    assert run(driver, "uncompress", abi.CODEC_GZIP, one, out) == ["U runtime_error"]
    # three bytes are not a whole zstd frame header: ZSTD_decompressStream
    # consumes them and asks for more, the reference loop ends with an empty
    # result (stream_zstd.cc:160-176)
    assert run(driver, "uncompress", abi.CODEC_ZSTD, one, out) == ["U ok 0"]
    import gzip
    from tests.test_hostcodec import corpus, zstd_compress
    gz, zs = str(tmp_path / "a.gz"), str(tmp_path / "a.zst")
    open(gz, "wb").write(gzip.compress(corpus(20, 200000)))
    open(zs, "wb").write(zstd_compress(corpus(21, 200000)))
    o1, o2 = str(tmp_path / "a.gz.out"), str(tmp_path / "a.zst.out")
    assert run(driver, "uncompress", abi.CODEC_GZIP, gz, o1, abi.CODEC_ZSTD, zs, o2) == ["U ok 200000"] * 2
    assert open(o1, "rb").read() == corpus(20, 200000) and open(o2, "rb").read() == corpus(21, 200000)


# ---------------------------------------------------------------------------
# GPU: kafka::batch_reader (wire layout)
# ---------------------------------------------------------------------------

def ref_batch_reader(rs: bytes, oracle):
    """kafka::batch_reader + kafka_batch_adapter::adapt over raw bytes
    (kafka/protocol/batch_reader.cc:50-156, kafka_batch_adapter.cc:32-188):
    the events surfaces_main.cpp prints."""
    def last_offset():
        pos, last = 0, 0
        while len(rs) - pos:
            if len(rs) - pos < 61:
                return "L corrupt"
            size = struct.unpack_from(">i", rs, pos + 8)[0] + 12
            if size < 61 or pos + size > len(rs):
                return "L out_of_range"
            base = struct.unpack_from(">q", rs, pos)[0]
            lod = struct.unpack_from(">i", rs, pos + 23)[0]
            last = base + lod
            pos += size
        return f"L {last}"

    ev = [last_offset()]
    pos = 0
    while len(rs) - pos:
        if len(rs) - pos < 61:
            ev.append("X corrupt")
            break
        size = struct.unpack_from(">i", rs, pos + 8)[0] + 12
        if size < 61 or pos + size > len(rs):
            ev.append("X out_of_range")
            break
        b = rs[pos:pos + size]
        v2 = b[16] == 2
        crc_ok = v2 and oracle.crc32c(b[21:]) == struct.unpack_from(">I", b, 17)[0]
        pos += size
        if not crc_ok:
            ev.append(f"B {int(v2)} 0 0")
            continue
        codec = struct.unpack_from(">h", b, 21)[0] & 7
        if codec > 4:
            ev.append("X runtime_error")
            break
        if codec == 0:
            rc = struct.unpack_from(">i", b, 57)[0]
            _, perr, trailing, _ = oracle.walk_records(b[61:], rc)
            if perr != 0 or trailing != 0:
                ev.append(f"B 1 1 0")
                continue
        base = struct.unpack_from(">q", b, 0)[0]
        ev.append(f"B 1 1 1 {base} {size} {size - 61} {oracle.crc32c(b[61:])}")
    return ev


@pytest.mark.gpu
def test_kafka_batch_reader(driver, rplib, oracle, engine, tmp_path):
    seg = gen(rplib, 300_000, 3, seed=0x5A, batch_bytes=0, min_batch=200, max_batch=30_000, corrupt_payload_ppm=100_000)
    rs = bg.disk_to_wire(seg.tobytes())
    cases = {"clean": rs}
    b = bytearray(rs)
    b[16 + bg.wire_batches(rs)[1][0]] = 1  # magic of batch 1
    cases["magic"] = bytes(b)
    p3, s3 = bg.wire_batches(rs)[3]
    cases["truncated"] = rs[: p3 + s3 - 9]
    cases["short_tail"] = rs[: p3 + s3 + 40]
    b = bytearray(rs)
    struct.pack_into(">i", b, p3 + 8, 10)
    cases["small_length"] = bytes(b)
    b = bytearray(rs)
    b[p3 + 22] = (b[p3 + 22] & ~7) | 5
    struct.pack_into(">I", b, p3 + 17, bg.crc32c(bytes(b[p3 + 21:p3 + s3])))
    cases["codec5"] = bytes(b)
    cases["empty"] = b""
    for name, data in cases.items():
        got = run(driver, "wire", write(tmp_path, name, data))
        assert got == ref_batch_reader(data, oracle), name


# ---------------------------------------------------------------------------
# GPU: the write side (storage::stamp_batches over rpgpu_stamp)
# ---------------------------------------------------------------------------
@pytest.mark.gpu
def test_stamp_batches_surface(driver, oracle, rplib, tmp_path):
    """storage::stamp_batches (disk_log_appender offsets + reset_size_checksum_
    metadata + header_crc) == the oracle, and returns the appender's next
    offset (last_offset + 1)."""
    import synth
    a = np.zeros(3 << 20, dtype=np.uint8)
    synth.gen_segment(a, 1, seed=0xC5, batch_bytes=0, min_batch=61, max_batch=400000, weights=[40, 0, 15, 30, 0, 15])
    r = oracle.run_job(a, [0, a.size], abi.JOB_CRC)
    b = r.batches
    end = int(b["file_pos"][-1]) + int(b["size_bytes"][-1])
    seg = a[:end].copy()
    pos = b["file_pos"].astype(np.uint64)
    pl = (b["size_bytes"] - abi.HEADER_SIZE).astype(np.uint32)
    for p in pos:
        seg[int(p):int(p) + 16] = 0
        seg[int(p) + 17:int(p) + 21] = 0
    src, posf, out = tmp_path / "in.bin", tmp_path / "pos.txt", tmp_path / "out.bin"
    seg.tofile(src)
    posf.write_text(" ".join(str(int(p)) for p in pos))
    lines = run(driver, "stamp", str(src), str(posf), str(out), "1000", str(abi.STAMP_OFFSETS | abi.STAMP_CRC))
    want = oracle.stamp_batches(seg, pos, pl, 1000, abi.STAMP_OFFSETS | abi.STAMP_CRC)
    got = np.fromfile(out, dtype=np.uint8)
    np.testing.assert_array_equal(got, want)
    nxt = 1000 + int(np.sum(b["last_offset_delta"].astype(np.int64) + 1))
    assert lines == [f"S {nxt}"]


@pytest.mark.gpu
@pytest.mark.parametrize("codec", [abi.CODEC_LZ4, abi.CODEC_SNAPPY])
def test_compress_batch_surface(driver, oracle, rplib, tmp_path, codec):
    """storage::internal::compress_batch (parser_utils.cc:96-111): the payload
    compressed (== the oracle's compressor), attrs gain the codec, size / crc
    / header_crc reset — the result validates and decodes back to the
    original records."""
    a = np.zeros(1 << 20, dtype=np.uint8)
    synth.gen_segment(a, 0, seed=0xC1, batch_bytes=0, min_batch=300000, max_batch=400000, weights=[1, 0, 0, 0, 0, 0])
    r = oracle.run_job(a, [0, a.size], abi.JOB_CRC | abi.JOB_PARSE)
    b = r.batches[0]
    p, sz = int(b["file_pos"]), int(b["size_bytes"])
    batch = a[p:p + sz].copy()
    src, out = tmp_path / "b.bin", tmp_path / "c.bin"
    batch.tofile(src)
    lines = run(driver, "compress_batch", codec, str(src), str(out))
    got = np.fromfile(out, dtype=np.uint8)
    payload = got[abi.HEADER_SIZE:].tobytes()
    assert payload == oracle.compress(codec, batch[abi.HEADER_SIZE:].tobytes())
    assert lines == [f"C {got.size} {len(payload)}"]
    seg = np.concatenate([got, np.zeros(64, np.uint8)])
    res = oracle.run_job(seg, [0, got.size], abi.JOB_CRC | abi.JOB_PARSE | abi.JOB_DECODE)
    rb = res.batches[0]
    assert rb["flags"] & abi.F_CRC_OK and rb["flags"] & abi.F_HEADER_OK and rb["flags"] & abi.F_CODEC_OK
    assert (int(rb["attrs"]) & 7) == codec and int(rb["base_offset"]) == int(b["base_offset"])
    assert int(rb["decoded_len"]) == sz - abi.HEADER_SIZE
