"""ctypes wrapper over the CPU oracle (liboracle.so) and the codec harness
(_ref/libcodecref.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — as the checker, never as the thing measured or
shipped.  The product (redpanda_amd) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from redpanda_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libcodecref.so")

_lib = None
_ref = None

u8p = C.POINTER(C.c_uint8)


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.rpo_crc32c_extend.restype = C.c_uint32
        L.rpo_crc32c_extend.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t]
        L.rpo_crc32c_extend_hw.restype = C.c_uint32
        L.rpo_crc32c_extend_hw.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t]
        L.rpo_crc32c_combine.restype = C.c_uint32
        L.rpo_crc32c_combine.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64]
        L.rpo_xxh32.restype = C.c_uint32
        L.rpo_xxh32.argtypes = [C.c_void_p, C.c_size_t, C.c_uint32]
        L.rpo_vint_deserialize.restype = C.c_int64
        L.rpo_vint_deserialize.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
        L.rpo_vint_serialize.restype = C.c_size_t
        L.rpo_vint_serialize.argtypes = [C.c_int64, C.c_void_p]
        for name in ("rpo_lz4f_uncompress", "rpo_snappy_raw_uncompress",
                     "rpo_snappy_java_uncompress"):
            f = getattr(L, name)
            f.restype = C.c_int
            f.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
        L.rpo_uncompress.restype = C.c_int
        L.rpo_uncompress.argtypes = [C.c_int, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                     C.POINTER(C.c_size_t)]
        L.rpo_lz4_block_decode.restype = C.c_int
        L.rpo_lz4_block_decode.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_size_t]
        L.rpo_decode_capacity.restype = C.c_uint64
        L.rpo_decode_capacity.argtypes = [C.c_int, C.c_void_p, C.c_size_t]
        L.rpo_walk_records.restype = C.c_uint32
        L.rpo_walk_records.argtypes = [C.c_void_p, C.c_size_t, C.c_int32, C.c_uint32, C.c_void_p,
                                       C.c_uint64, C.POINTER(C.c_uint8), C.POINTER(C.c_uint64)]
        L.rpo_run_job.restype = C.c_int
        L.rpo_run_job.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p,
                                  C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                  C.c_void_p, C.c_void_p, C.c_void_p]
        L.rpo_run_job_layout.restype = C.c_int
        L.rpo_run_job_layout.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                         C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                         C.c_void_p, C.c_void_p, C.c_void_p]
        L.rpo_batch_valid.restype = C.c_int
        L.rpo_batch_valid.argtypes = [C.c_void_p, C.c_uint32]
        L.rpo_baseline_validate.restype = C.c_int64
        L.rpo_baseline_validate.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int, C.c_int,
                                            C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
        L.rpo_stamp_batches.restype = None
        L.rpo_stamp_batches.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int64, C.c_uint32]
        for name in ("rpo_lz4f_compress_bound",):
            getattr(L, name).restype = C.c_size_t
            getattr(L, name).argtypes = [C.c_size_t]
        L.rpo_snappy_java_compress_bound.restype = C.c_size_t
        L.rpo_snappy_java_compress_bound.argtypes = [C.c_size_t, C.c_size_t]
        L.rpo_lz4f_compress.restype = C.c_size_t
        L.rpo_lz4f_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
        L.rpo_snappy_java_compress.restype = C.c_size_t
        L.rpo_snappy_java_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p]
        L.rpo_segment_index.restype = C.c_int
        L.rpo_serialize_wire.restype = C.c_uint64
        L.rpo_serialize_wire.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p]
        L.rpo_segment_index.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_uint64,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


def ref():
    """liblz4 1.9.3 / libsnappy 1.1.8 harness, or None when not buildable."""
    global _ref
    if _ref is None:
        if not os.path.exists(REF_PATH):
            try:
                build()
            except Exception:
                return None
        if not os.path.exists(REF_PATH):
            return None
        R = C.CDLL(REF_PATH)
        for name in ("ref_lz4f_uncompress", "ref_snappy_raw", "ref_snappy_java"):
            f = getattr(R, name)
            f.restype = C.c_int
            f.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
        R.ref_lz4_block.restype = C.c_int
        R.ref_lz4_block.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        R.ref_lz4f_compress.restype = C.c_size_t
        R.ref_lz4f_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int,
                                        C.c_int, C.c_int, C.c_int, C.c_int]
        R.ref_lz4f_bound.restype = C.c_size_t
        R.ref_lz4f_bound.argtypes = [C.c_size_t]
        R.ref_snappy_compress.restype = C.c_size_t
        R.ref_snappy_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        R.ref_snappy_bound.restype = C.c_size_t
        R.ref_snappy_bound.argtypes = [C.c_size_t]
        R.ref_lz4f_compress_stream.restype = C.c_size_t
        R.ref_lz4f_compress_stream.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p, C.c_size_t]
        R.ref_snappy_java_compress.restype = C.c_size_t
        R.ref_snappy_java_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p, C.c_size_t]
        R.ref_baseline_decode.restype = C.c_double
        R.ref_baseline_decode.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.POINTER(C.c_uint64),
                                          C.POINTER(C.c_uint64)]
        _ref = R
    return _ref


def _buf(b):
    if isinstance(b, np.ndarray):
        return b.ctypes.data_as(C.c_void_p), b.nbytes
    b = bytes(b)
    return C.cast(C.c_char_p(b), C.c_void_p), len(b)


def crc32c(data: bytes, crc: int = 0) -> int:
    """google crc32c::Extend(crc, data) — the standard CRC32C when crc == 0."""
    arr = np.frombuffer(bytes(data), dtype=np.uint8)
    return lib().rpo_crc32c_extend(crc, arr.ctypes.data_as(C.c_void_p), arr.size)


def crc32c_hw(data: bytes, crc: int = 0) -> int:
    arr = np.frombuffer(bytes(data), dtype=np.uint8)
    return lib().rpo_crc32c_extend_hw(crc, arr.ctypes.data_as(C.c_void_p), arr.size)


def xxh32(data: bytes, seed: int = 0) -> int:
    arr = np.frombuffer(bytes(data), dtype=np.uint8)
    return lib().rpo_xxh32(arr.ctypes.data_as(C.c_void_p), arr.size, seed)


def vint_deserialize(data: bytes):
    arr = np.frombuffer(bytes(data) + b"\0", dtype=np.uint8)
    br = C.c_size_t(0)
    v = lib().rpo_vint_deserialize(arr.ctypes.data_as(C.c_void_p), len(data), C.byref(br))
    return v, br.value


def vint_serialize(v: int) -> bytes:
    out = (C.c_uint8 * 10)()
    n = lib().rpo_vint_serialize(v, out)
    return bytes(out[:n])


def _codec_call(fn, data: bytes, cap: int):
    src = np.frombuffer(bytes(data) + b"\0" * 8, dtype=np.uint8)
    dst = np.zeros(max(cap, 1), dtype=np.uint8)
    out = C.c_size_t(0)
    rc = fn(src.ctypes.data_as(C.c_void_p), len(data), dst.ctypes.data_as(C.c_void_p), cap, C.byref(out))
    return rc, bytes(dst[: out.value]) if rc == 0 else b""


def uncompress(codec: int, data: bytes, cap: int = None):
    """(rc, bytes): rc 0 ok, -1 reference throws, -2 capacity too small."""
    if cap is None:
        cap = max(decode_capacity(codec, data), 1)
    return _codec_call(lambda s, n, d, c, o: lib().rpo_uncompress(codec, s, n, d, c, o), data, cap)


def lz4f_uncompress(data: bytes, cap: int):
    return _codec_call(lib().rpo_lz4f_uncompress, data, cap)


def snappy_java_uncompress(data: bytes, cap: int):
    return _codec_call(lib().rpo_snappy_java_uncompress, data, cap)


def snappy_raw_uncompress(data: bytes, cap: int):
    return _codec_call(lib().rpo_snappy_raw_uncompress, data, cap)


def lz4_block_decode(data: bytes, cap: int, history: bytes = b""):
    src = np.frombuffer(bytes(data) + b"\0" * 8, dtype=np.uint8)
    dst = np.zeros(len(history) + cap + 64, dtype=np.uint8)
    dst[: len(history)] = np.frombuffer(history, dtype=np.uint8)
    p = dst.ctypes.data + len(history)
    r = lib().rpo_lz4_block_decode(src.ctypes.data_as(C.c_void_p), len(data), C.c_void_p(p), cap,
                                   len(history))
    return r, bytes(dst[len(history): len(history) + max(r, 0)])


def decode_capacity(codec: int, data: bytes) -> int:
    src = np.frombuffer(bytes(data) + b"\0" * 8, dtype=np.uint8)
    return lib().rpo_decode_capacity(codec, src.ctypes.data_as(C.c_void_p), len(data))


def walk_records(payload: bytes, record_count: int, batch: int = 0, cap: int = None):
    src = np.frombuffer(bytes(payload) + b"\0" * 16, dtype=np.uint8)
    if cap is None:
        cap = max(record_count, 0)
    idx = np.zeros(max(cap, 1), dtype=abi.RECORD_INDEX)
    perr = C.c_uint8(0)
    trailing = C.c_uint64(0)
    n = lib().rpo_walk_records(src.ctypes.data_as(C.c_void_p), len(payload), record_count, batch,
                               idx.ctypes.data_as(C.c_void_p), cap, C.byref(perr), C.byref(trailing))
    return n, perr.value, trailing.value, idx[: min(n, cap)]


class JobResult:
    def __init__(self, batches, records, decoded, summaries, totals, bitmap):
        self.batches = batches
        self.records = records
        self.decoded = decoded
        self.summaries = summaries
        self.totals = totals
        self.bitmap = bitmap


def run_job(data: np.ndarray, seg_offsets, flags=abi.JOB_CRC | abi.JOB_PARSE | abi.JOB_DECODE,
            batch_cap=None, record_cap=None, decoded_cap=None, layout: int = abi.LAYOUT_DISK) -> JobResult:
    """Oracle run of the rpgpu_job contract over host-resident segments
    (layout: abi.LAYOUT_DISK segments or abi.LAYOUT_WIRE Kafka record sets)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offs = np.ascontiguousarray(np.asarray(seg_offsets, dtype=np.uint64))
    nseg = offs.size - 1
    total = int(offs[-1])
    if batch_cap is None:
        batch_cap = total // abi.HEADER_SIZE + nseg + 1
    if record_cap is None:
        record_cap = max(total // 2, 16)
    if decoded_cap is None:
        decoded_cap = max(total * 64, 1 << 16)
    batches = np.zeros(batch_cap, dtype=abi.BATCH_RESULT)
    records = np.zeros(max(record_cap, 1), dtype=abi.RECORD_INDEX)
    decoded = np.zeros(max(decoded_cap, 1), dtype=np.uint8)
    summaries = np.zeros(max(nseg, 1), dtype=abi.SEGMENT_SUMMARY)
    totals = np.zeros(1, dtype=abi.JOB_TOTALS)
    bitmap = np.zeros(batch_cap // 64 + 1, dtype=np.uint64)
    pad = np.zeros(data.size + 64, dtype=np.uint8)
    pad[: data.size] = data
    lib().rpo_run_job_layout(pad.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p), nseg, flags, layout,
                      batches.ctypes.data_as(C.c_void_p), batch_cap,
                      records.ctypes.data_as(C.c_void_p), record_cap,
                      decoded.ctypes.data_as(C.c_void_p), decoded_cap,
                      summaries.ctypes.data_as(C.c_void_p), totals.ctypes.data_as(C.c_void_p),
                      bitmap.ctypes.data_as(C.c_void_p))
    nb = int(totals[0]["n_batches"])
    nr = int(totals[0]["n_records"])
    nd = int(totals[0]["decoded_bytes"])
    return JobResult(batches[:nb], records[:nr], decoded[:nd], summaries[:nseg], totals[0],
                     bitmap[: (nb + 63) // 64])


def baseline_validate(data: np.ndarray, seg_offsets, threads: int, hw: bool = True):
    offs = np.ascontiguousarray(np.asarray(seg_offsets, dtype=np.uint64))
    secs = C.c_double(0)
    nbytes = C.c_uint64(0)
    nb = lib().rpo_baseline_validate(data.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p),
                                     offs.size - 1, threads, 1 if hw else 0, C.byref(secs),
                                     C.byref(nbytes))
    return nb, secs.value, nbytes.value


def baseline_decode(seg: np.ndarray, positions, threads: int):
    """CPU baseline of the decode path over the batches at `positions` of
    `seg` (stored crc + liblz4/libsnappy uncompress + decoded crc, one
    pthread per core): (seconds, stored bytes, decoded bytes)."""
    R = ref()
    if R is None:
        raise RuntimeError("codec harness (oracle/_ref/libcodecref.so) not built")
    pos = np.ascontiguousarray(np.asarray(positions, dtype=np.uint64))
    s, d = C.c_uint64(0), C.c_uint64(0)
    secs = R.ref_baseline_decode(seg.ctypes.data_as(C.c_void_p), pos.ctypes.data_as(C.c_void_p), pos.size, threads,
                                 C.byref(s), C.byref(d))
    return secs, s.value, d.value


def serialize_wire(data: np.ndarray, seg_offsets, batches: np.ndarray, first: int = 0, n: int = None) -> bytes:
    """kafka::writer_serialize_batch (kafka/protocol/response_writer.h:241-276)
    over batches [first, first + n) of a job's results."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offs = np.ascontiguousarray(np.asarray(seg_offsets, dtype=np.uint64))
    b = np.ascontiguousarray(batches, dtype=abi.BATCH_RESULT)
    n = b.size - first if n is None else n
    args = (data.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p), b.ctypes.data_as(C.c_void_p), first, n)
    size = lib().rpo_serialize_wire(*args, None)
    out = np.zeros(max(size, 1), dtype=np.uint8)
    lib().rpo_serialize_wire(*args, out.ctypes.data_as(C.c_void_p))
    return out[:size].tobytes()


def segment_index(batches: np.ndarray, summaries: np.ndarray, base_offsets, step: int = abi.INDEX_DEFAULT_STEP,
                  batch_cap: int = None):
    """Oracle: segment_index::maybe_track replayed over each segment's
    crc-good prefix (storage/log_replayer.cc:62-74, storage/segment_index.cc:58-72,
    storage/index_state.cc:48-95).  Same per-segment output as
    Engine.index_to_host: [(index_state row, relative_offset, relative_time, position)]."""
    batches = np.ascontiguousarray(batches, dtype=abi.BATCH_RESULT)
    summaries = np.ascontiguousarray(summaries, dtype=abi.SEGMENT_SUMMARY)
    nseg = summaries.size
    cap = batches.size if batch_cap is None else batch_cap
    bb = np.zeros(max(cap, 1), dtype=abi.BATCH_RESULT)
    bb[: min(cap, batches.size)] = batches[:cap]
    st = np.zeros(max(nseg, 1), dtype=abi.INDEX_STATE)
    st["base_offset"][:nseg] = np.asarray(base_offsets, dtype=np.int64)
    ro = np.zeros(max(cap, 1), dtype=np.uint32)
    rt = np.zeros(max(cap, 1), dtype=np.uint32)
    ps = np.zeros(max(cap, 1), dtype=np.uint64)
    rc = lib().rpo_segment_index(bb.ctypes.data_as(C.c_void_p), cap, summaries.ctypes.data_as(C.c_void_p), nseg,
                                 step, st.ctypes.data_as(C.c_void_p), ro.ctypes.data_as(C.c_void_p),
                                 rt.ctypes.data_as(C.c_void_p), ps.ctypes.data_as(C.c_void_p))
    if rc != 0:
        raise RuntimeError(f"rpo_segment_index: {rc}")
    out = []
    for s in st[:nseg]:
        a, n = int(s["first_entry"]), int(s["n_entries"])
        out.append((s, ro[a:a + n].copy(), rt[a:a + n].copy(), ps[a:a + n].copy()))
    return out


def stamp_batches(data: np.ndarray, positions, payload_lens, next_offset: int = 0, flags: int = 3) -> np.ndarray:
    """Oracle of the write side (rpgpu_stamp): a stamped copy of `data`
    (disk_log_appender::operator() + reset_size_checksum_metadata, in batch
    order; flags 1 = offsets, 2 = size + crc; header_crc always)."""
    out = np.array(data, dtype=np.uint8, copy=True)
    pos = np.ascontiguousarray(np.asarray(positions, dtype=np.uint64))
    pl = np.ascontiguousarray(np.asarray(payload_lens, dtype=np.uint32))
    lib().rpo_stamp_batches(out.ctypes.data, pos.ctypes.data, pl.ctypes.data, len(pos), next_offset, flags)
    return out


def compress(codec: int, data: bytes, frag: int = 0) -> bytes:
    """Oracle of the write side's compressor::compress (rp_oracle.c):
    codec 3 = lz4 frame (lz4_frame_compressor.cc:72-113), 2 = snappy-java
    over `frag`-byte iobuf fragments (snappy_java_compressor.cc:58-75)."""
    src = np.frombuffer(bytes(data), dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    L = lib()
    if codec == 3:
        out = np.zeros(L.rpo_lz4f_compress_bound(len(data)), np.uint8)
        n = L.rpo_lz4f_compress(src.ctypes.data, len(data), out.ctypes.data)
    elif codec == 2:
        out = np.zeros(L.rpo_snappy_java_compress_bound(len(data), frag), np.uint8)
        n = L.rpo_snappy_java_compress(src.ctypes.data, len(data), frag, out.ctypes.data)
    else:
        raise ValueError(codec)
    return out[:n].tobytes()


def ref_compress(codec: int, data: bytes, frag: int = 0):
    """The same through the reference's codec libraries (oracle/_ref), or
    None when the harness is absent."""
    R = ref()
    if R is None:
        return None
    src = np.frombuffer(bytes(data), dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    cap = 2 * len(data) + (256 << 10)
    out = np.zeros(cap, np.uint8)
    f = R.ref_lz4f_compress_stream if codec == 3 else R.ref_snappy_java_compress
    n = f(src.ctypes.data, len(data), frag, out.ctypes.data, cap)
    assert n > 0
    return out[:n].tobytes()
