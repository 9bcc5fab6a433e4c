"""Synthetic segment generator (test and benchmark data; NOT the product).

librpgen.so builds seeded Redpanda segments after the reference's test batch
recipe (storage/tests/utils/random_batch.cc:50-154) and compresses payloads
with the reference's own codec libraries.  tests/, bench.py and
__graft_entry__.smoke() load it; redpanda_amd never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librpgen.so")
SRC = os.path.join(HERE, "rp_gen.cpp")
HDR = os.path.join(HERE, "rpgen.h")
CONDA = "/opt/conda"

# rpgen_codec_slot
NONE, GZIP, SNAPPY_JAVA, LZ4, ZSTD, SNAPPY_RAW = range(6)
SLOTS = 6

_lib = None


class SpecC(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64), ("segment_bytes", C.c_uint64), ("batch_bytes", C.c_uint32),
        ("min_batch_bytes", C.c_uint32), ("max_batch_bytes", C.c_uint32), ("value_bytes", C.c_uint32),
        ("key_bytes", C.c_uint32), ("headers_per_record", C.c_uint32), ("codec_weights", C.c_uint32 * SLOTS),
        ("lz4_linked_ppm", C.c_uint32), ("lz4_content_checksum_ppm", C.c_uint32),
        ("lz4_block_checksum_ppm", C.c_uint32), ("corrupt_ppm_payload", C.c_uint32),
        ("corrupt_ppm_header", C.c_uint32), ("corrupt_ppm_zero", C.c_uint32), ("truncate_tail", C.c_uint32),
        ("size_uniform", C.c_uint32), ("base_offset", C.c_int64),
    ]


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or \
            os.path.getmtime(LIB_PATH) < max(os.path.getmtime(SRC), os.path.getmtime(HDR)):
        cmd = ["g++", "-O2", "-fPIC", "-std=c++17", "-Wall", "-shared", "-I", HERE, "-I", f"{CONDA}/include", SRC,
               "-o", LIB_PATH, "-L", f"{CONDA}/lib", f"-Wl,-rpath,{CONDA}/lib", "-llz4", "-lsnappy", "-lz", "-lzstd",
               "-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("librpgen build failed:\n" + r.stdout + r.stderr)
    return LIB_PATH


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.rpgen_segment.restype = C.c_int64
        L.rpgen_segment.argtypes = [C.POINTER(SpecC), C.c_uint32, C.c_void_p]
        L.rpgen_crc32c.restype = C.c_uint32
        L.rpgen_crc32c.argtypes = [C.c_uint32, C.c_void_p, C.c_uint64]
        _lib = L
    return _lib


def gen_segment(out, segment_index: int, *, seed: int, batch_bytes: int = 16384, min_batch: int = 0,
                max_batch: int = 0, value_bytes: int = 1024, key_bytes: int = 16, headers: int = 2,
                codec_mix: int = 1, weights=None, lz4_linked_ppm: int = 0, lz4_content_checksum_ppm: int = 0,
                lz4_block_checksum_ppm: int = 0, corrupt_payload_ppm: int = 0, corrupt_header_ppm: int = 0,
                corrupt_zero_ppm: int = 0, truncate_tail: bool = False, size_uniform: bool = False,
                base_offset: int = 0) -> int:
    """Fill the numpy uint8 array `out` with one seeded segment; returns the
    number of whole batches.  `weights` = relative weights per codec slot
    (NONE, GZIP, SNAPPY_JAVA, LZ4, ZSTD, SNAPPY_RAW); without it `codec_mix`
    (bitmask of 1 << codec) gives equal weights to the codecs it names."""
    if weights is None:
        weights = [1 if codec_mix & (1 << c) else 0 for c in range(5)] + [0]
    w = (C.c_uint32 * SLOTS)(*[int(x) for x in list(weights) + [0] * (SLOTS - len(weights))])
    spec = SpecC(seed=seed, segment_bytes=out.nbytes, batch_bytes=batch_bytes, min_batch_bytes=min_batch,
                 max_batch_bytes=max_batch, value_bytes=value_bytes, key_bytes=key_bytes, headers_per_record=headers,
                 codec_weights=w, lz4_linked_ppm=lz4_linked_ppm, lz4_content_checksum_ppm=lz4_content_checksum_ppm,
                 lz4_block_checksum_ppm=lz4_block_checksum_ppm, corrupt_ppm_payload=corrupt_payload_ppm,
                 corrupt_ppm_header=corrupt_header_ppm, corrupt_ppm_zero=corrupt_zero_ppm,
                 truncate_tail=1 if truncate_tail else 0,
                 size_uniform=1 if size_uniform else 0, base_offset=base_offset)
    n = load().rpgen_segment(C.byref(spec), segment_index, out.ctypes.data_as(C.c_void_p))
    if n < 0:
        raise RuntimeError(f"rpgen_segment failed: {n}")
    return n


def crc32c(data, crc: int = 0) -> int:
    import numpy as np
    a = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data)
    return load().rpgen_crc32c(crc, a.ctypes.data_as(C.c_void_p), a.nbytes)


# SURVEY.md §8(d) recipes (kwargs of gen_segment)
C1 = dict(seed=0xC1)
C2 = dict(seed=0xC2, batch_bytes=0, min_batch=64 << 10, max_batch=1 << 20, weights=[0, 0, 0, 1, 0, 0],
          size_uniform=True, lz4_linked_ppm=100000, lz4_content_checksum_ppm=100000)
C5 = dict(seed=0xC5, batch_bytes=0, min_batch=200, max_batch=1 << 20, weights=[40, 0, 15, 30, 0, 15],
          corrupt_payload_ppm=10000, corrupt_header_ppm=2000, corrupt_zero_ppm=1000, truncate_tail=True)
# C5 with 10% gzip and 10% zstd: both decoded on the
# device (zstd through the host with RPGPU_JOB_HOST_CODECS)
C6 = dict(seed=0xC6, batch_bytes=0, min_batch=200, max_batch=1 << 20, weights=[32, 10, 12, 24, 10, 12],
          corrupt_payload_ppm=10000, corrupt_header_ppm=2000, corrupt_zero_ppm=1000, truncate_tail=True)
