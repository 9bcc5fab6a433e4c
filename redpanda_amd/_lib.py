"""ctypes binding of librpgpu.so (the C-ABI in include/rpgpu.h).

The HIP path is the only path: if the library is missing, or a GPU entry
point is called without a device, this raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import re

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librpgpu.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "rpgpu.h")

_lib = None


class RpgpuError(RuntimeError):
    pass


class JobC(C.Structure):
    _fields_ = [
        ("d_data", C.c_void_p), ("d_seg_offsets", C.c_void_p), ("h_seg_offsets", C.c_void_p),
        ("n_segments", C.c_uint32), ("layout", C.c_uint32), ("flags", C.c_uint32),
        ("chunk_bytes", C.c_uint32),
        ("d_batches", C.c_void_p), ("batch_capacity", C.c_uint64),
        ("d_records", C.c_void_p), ("record_capacity", C.c_uint64),
        ("d_decoded", C.c_void_p), ("decoded_capacity", C.c_uint64),
        ("d_summaries", C.c_void_p), ("d_totals", C.c_void_p), ("d_valid_bitmap", C.c_void_p),
        ("d_seeds", C.c_void_p), ("d_seed_offsets", C.c_void_p),
    ]


class CapacityC(C.Structure):
    """rpgpu_capacity (include/rpgpu.h)."""
    _fields_ = [("n_batches", C.c_uint64), ("record_capacity", C.c_uint64), ("decoded_capacity", C.c_uint64),
                ("reserved", C.c_uint64)]


def exported_symbols_from_header(path: str = HEADER):
    """Function names declared in include/rpgpu.h."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(rpgpu_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def load():
    """Load librpgpu.so.  When torch is importable it is imported first so the
    process has exactly one HIP runtime (torch bundles libamdhip64.so.7)."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401  (one HIP runtime per process)
    except Exception:
        pass
    path = LIB_PATH
    if os.environ.get("RPGPU_CHECKED") == "1":
        path = os.path.join(HERE, "librpgpu_checked.so")
    elif os.environ.get("RPGPU_STAMPS") == "1":
        path = os.path.join(HERE, "librpgpu_stamps.so")
    elif os.environ.get("RPGPU_VARIANT"):
        # experiment builds (scripts/build_exp.py): librpgpu_<variant>.so
        path = os.path.join(HERE, f"librpgpu_{os.environ['RPGPU_VARIANT']}.so")
    if not os.path.exists(path):
        raise RpgpuError(f"{path} missing: run `python -m redpanda_amd.build` (no CPU fallback exists)")
    L = C.CDLL(path)
    vp, i32, u32, u64, sz = C.c_void_p, C.c_int, C.c_uint32, C.c_uint64, C.c_size_t
    sig = {
        "rpgpu_device_count": (i32, []),
        "rpgpu_create": (i32, [i32, C.POINTER(vp)]),
        "rpgpu_destroy": (i32, [vp]),
        "rpgpu_strerror": (C.c_char_p, [i32]),
        "rpgpu_last_error": (C.c_char_p, [vp]),
        "rpgpu_dev_alloc": (i32, [vp, sz, C.POINTER(vp)]),
        "rpgpu_dev_free": (i32, [vp, vp]),
        "rpgpu_host_alloc": (i32, [vp, sz, C.POINTER(vp)]),
        "rpgpu_host_free": (i32, [vp, vp]),
        "rpgpu_memcpy_h2d": (i32, [vp, vp, vp, sz, vp]),
        "rpgpu_memcpy_d2h": (i32, [vp, vp, vp, sz, vp]),
        "rpgpu_memset": (i32, [vp, vp, i32, sz, vp]),
        "rpgpu_sync": (i32, [vp, vp]),
        "rpgpu_crc32c_extend": (u32, [u32, vp, sz]),
        "rpgpu_submit": (i32, [vp, C.POINTER(JobC), vp]),
        "rpgpu_last_timings": (i32, [vp, C.POINTER(C.c_float), i32]),
        "rpgpu_set_timing": (i32, [vp, i32]),
        "rpgpu_uncompress": (i32, [vp, i32, vp, sz, vp, sz, C.POINTER(sz)]),
        "rpgpu_uncompress_batch": (i32, [vp, u32, vp, vp, vp, vp, vp, vp, vp]),
        "rpgpu_compress_batch": (i32, [vp, u32, vp, vp, vp, vp, vp, vp, vp, vp]),
        "rpgpu_compress_bound": (C.c_size_t, [C.c_int, C.c_size_t, C.c_size_t]),
        "rpgpu_submit_async": (i32, [vp, C.POINTER(JobC), vp, C.POINTER(vp)]),
        "rpgpu_poll": (i32, [vp]),
        "rpgpu_wait": (i32, [vp]),
        "rpgpu_release": (i32, [vp]),
        "rpgpu_query_capacity": (i32, [vp, C.POINTER(JobC), vp, C.POINTER(CapacityC)]),
        "rpgpu_stamp": (i32, [vp, vp, vp, vp, u32, C.c_int64, u32, vp]),
        "rpgpu_serialize_wire": (i32, [vp, vp, vp, vp, u64, u32, vp, vp, vp]),
        "rpgpu_validate_host": (i32, [vp, vp]),
        "rpgpu_segment_index": (i32, [vp, vp, u64, vp, u32, u64, vp, vp, vp, vp, vp]),
        "rpgpu_uncompress_bound": (u64, [i32, vp, sz]),
        "rpgpu_stamp_host": (i32, [vp, vp, sz, vp, vp, u32, C.c_int64, u32]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(rc: int, ctx=None, what: str = ""):
    if rc != 0:
        L = load()
        msg = L.rpgpu_strerror(rc).decode()
        if ctx is not None:
            detail = L.rpgpu_last_error(ctx)
            if detail:
                msg += f" ({detail.decode()})"
        raise RpgpuError(f"{what}: {msg} [{rc}]")


def crc32c(data, crc: int = 0) -> int:
    """crc::crc32c extend semantics (hashing/crc32c.h:19-40)."""
    import numpy as np
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    a = np.ascontiguousarray(a)
    return load().rpgpu_crc32c_extend(crc, a.ctypes.data_as(C.c_void_p), a.nbytes)


__all__ = ["load", "check", "crc32c", "JobC", "CapacityC", "RpgpuError", "abi",
           "exported_symbols_from_header"]
