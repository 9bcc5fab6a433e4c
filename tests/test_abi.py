"""The C-ABI library loads and exports every symbol include/rpgpu.h declares
(no compute calls: these run without a GPU).  Also: the host-side pieces of
the product that need no device (crc::crc32c host path, generator)."""
import ctypes as C
import os
import subprocess

import numpy as np

from redpanda_amd import abi
import synth  # noqa: E402  (test/bench data generator, not the product)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_every_declared_symbol_is_exported(rplib):
    L = rplib.load()
    names = rplib.exported_symbols_from_header()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", rplib.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert f" T {n}\n" in out or f" W {n}\n" in out, n


def test_struct_layouts_match_header():
    src = r'''
#include "rpgpu.h"
#include <stddef.h>
#include <stdio.h>
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(rpgpu_batch_result), sizeof(rpgpu_record_index),
         sizeof(rpgpu_segment_summary), sizeof(rpgpu_job_totals), offsetof(rpgpu_batch_result, flags),
         offsetof(rpgpu_record_index, end_pos), offsetof(rpgpu_job, d_valid_bitmap));
  return 0;
}'''
    exe = "/tmp/rpgpu_layout_check"
    r = subprocess.run(["gcc", "-x", "c", "-", "-I", os.path.join(ROOT, "include"), "-o", exe], input=src,
                       text=True, capture_output=True)
    assert r.returncode == 0, r.stderr
    vals = [int(x) for x in subprocess.run([exe], capture_output=True, text=True).stdout.split()]
    assert vals[:4] == [abi.BATCH_RESULT.itemsize, abi.RECORD_INDEX.itemsize, abi.SEGMENT_SUMMARY.itemsize,
                        abi.JOB_TOTALS.itemsize]
    assert vals[4] == abi.BATCH_RESULT.fields["flags"][1]
    assert vals[5] == abi.RECORD_INDEX.fields["end_pos"][1]
    from redpanda_amd._lib import JobC
    assert vals[6] == JobC.d_valid_bitmap.offset


def test_host_crc32c_surface(rplib, oracle):
    """crc::crc32c (hashing/crc32c.h) host path == oracle, incl. extend."""
    rnd = np.random.default_rng(1)
    for n in (0, 1, 3, 8, 57, 1000, 65537):
        d = rnd.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert rplib.crc32c(d) == oracle.crc32c(d)
        assert rplib.crc32c(d, 0x12345678) == oracle.crc32c(d, 0x12345678)
    assert rplib.crc32c(b"123456789") == 0xE3069283


def test_no_device_entry_points_fail_loudly(rplib):
    L = rplib.load()
    if L.rpgpu_device_count() > 0:
        return
    ctx = C.c_void_p()
    assert L.rpgpu_create(0, C.byref(ctx)) == -2  # RPGPU_E_NO_DEVICE: no CPU fallback


def test_generator_segments_validate_in_oracle(rplib, oracle):
    a = np.zeros(2 << 20, dtype=np.uint8)
    n = synth.gen_segment(a, 0, seed=0xC1)
    assert n == 128
    r = oracle.run_job(a, [0, a.size], abi.JOB_CRC | abi.JOB_PARSE)
    assert len(r.batches) == n
    assert np.all(r.batches["size_bytes"] == 16384)
    assert np.all(r.batches["flags"] == (abi.F_HEADER_OK | abi.F_COMPLETE | abi.F_CRC_OK | abi.F_PARSED |
                                         abi.F_PARSE_ASYNC_OK | abi.F_PARSE_OK | abi.F_INDEX_WRITTEN))
    b = np.zeros_like(a)
    synth.gen_segment(b, 0, seed=0xC1)
    assert np.array_equal(a, b)  # seeded: reproducible


def test_generator_codec_mix_decodes(rplib, oracle):
    a = np.zeros(4 << 20, dtype=np.uint8)
    synth.gen_segment(a, 2, seed=0xC2, batch_bytes=0, min_batch=64 << 10, max_batch=1 << 20,
                      codec_mix=(1 << abi.CODEC_LZ4) | (1 << abi.CODEC_SNAPPY))
    r = oracle.run_job(a, [0, a.size])
    f = r.batches["flags"]
    assert np.all(f & abi.F_COMPRESSED) and np.all(f & abi.F_CODEC_OK) and np.all(f & abi.F_PARSE_OK)
