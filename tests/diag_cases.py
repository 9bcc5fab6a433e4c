"""Cases that need the diagnostic library variant (librpgpu_diag.so, built by
__graft_entry__.build(); environment overrides of pool sizes and of the host
codec's availability).  A process loads one librpgpu, so tests/test_gpu_diag.py
runs each case here in a child process with RPGPU_VARIANT=diag:

    python -m tests.diag_cases <case>

exit status 0 = the case held; anything else prints why.
"""
import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from redpanda_amd import abi  # noqa: E402

DFLAGS = abi.JOB_CRC | abi.JOB_PARSE | abi.JOB_DECODE


def _gzip_payloads():
    """Clean gzip members of several sizes plus members whose ISIZE trailer
    claims ~4 GiB (the first pass's slot guess is payload-controlled)."""
    from tests import batchgen as BG
    from tests.gzip_corpus import gzip_member
    good = [gzip_member(BG.simple_records(n, vlen=v, seed=n), 6, 0) for n, v in
            [(5, 20), (40, 100), (300, 400), (900, 900), (60, 2000)]]
    hostile = []
    for p in good[1:4]:
        q = bytearray(p)
        q[-4:] = struct.pack("<I", 0xFFFFFFF0)
        hostile.append(bytes(q))
    return good[:2] + hostile[:1] + good[2:] + hostile[1:] + good


def case_small_pool():
    """RPGPU_INF_POOL_KIB=64: most members get no first-pass slot (and the
    hostile ISIZE ones are capped), so they decode in the second pass; every
    output is still the oracle's."""
    from oracle import oracle as O
    from redpanda_amd.engine import Engine
    from tests.test_gpu_parity import _gzip_batches, assert_same, run_both
    assert os.environ.get("RPGPU_INF_POOL_KIB"), "run with RPGPU_INF_POOL_KIB"
    O.build()
    eng = Engine(0)
    pay = _gzip_payloads()
    segs = [_gzip_batches(pay), _gzip_batches(pay[::-1], base=5000)]
    got, ref = run_both(eng, O, segs, flags=DFLAGS)
    ok = (got.batches["flags"] & abi.F_CODEC_OK) != 0
    assert int(np.sum(ok)) >= 2 * 8, int(np.sum(ok))
    assert_same(got, ref, DFLAGS)
    print(f"small_pool ok: {len(got.batches)} batches, {int(np.sum(ok))} decoded")


def case_host_codec_missing():
    """RPGPU_HOST_CODEC_MISSING=1: with RPGPU_JOB_HOST_CODECS a job holding
    zstd batches fails with RPGPU_E_UNSUPPORTED (valid payloads are never
    reported corrupt); without the flag the device decodes them."""
    import torch
    from oracle import oracle as O
    from redpanda_amd._lib import RpgpuError
    from redpanda_amd.engine import Engine
    from tests.test_gpu_parity import assert_same, gen, run_both
    assert os.environ.get("RPGPU_HOST_CODEC_MISSING") == "1"
    O.build()
    eng = Engine(0)
    segs = [gen(None, 1 << 20, i, seed=0x2E0 + i, batch_bytes=0, min_batch=200, max_batch=200000,
                weights=[1, 0, 0, 1, 3, 0]) for i in range(2)]
    data = np.concatenate(segs)
    offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
    d = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).cuda()[: data.size]
    try:
        eng.validate(d, offs, DFLAGS | abi.JOB_HOST_CODECS)
    except RpgpuError as e:
        assert f"[{abi.E_UNSUPPORTED}]" in str(e), e
    else:
        raise AssertionError("a host-codec job without libzstd must fail with RPGPU_E_UNSUPPORTED")
    got, ref = run_both(eng, O, segs, flags=DFLAGS)
    assert np.any(((got.batches["attrs"] & 7) == abi.CODEC_ZSTD) & ((got.batches["flags"] & abi.F_CODEC_OK) != 0))
    assert_same(got, ref, DFLAGS)
    print("host_codec_missing ok")


def case_small_frec():
    """RPGPU_FREC_CAP=n: the fast-path record pool holds n records, so the
    planner lists the first groups of LZ4 blocks for k_lzf_walk and leaves
    every later group (note_fast: no room) to k_lz_walk / k_lz_exec; frames
    mix listed blocks with walked ones.  Every field is still the oracle's
    (rp_codec.hip note_fast)."""
    import random
    import synth
    from oracle import oracle as O
    from redpanda_amd.engine import Engine
    from tests import test_gpu_lz4_walk as W
    from tests.test_gpu_parity import assert_same, gen, run_both
    assert os.environ.get("RPGPU_FREC_CAP"), "run with RPGPU_FREC_CAP"
    O.build()
    eng = Engine(0)
    rnd = random.Random(11)
    frames = []
    for kind in ("mixed", "text", "long_lits", "long_match"):
        for _ in range(3):
            blk, _ = W.valid_block(rnd, kind)
            frames.append(W.frame([blk]))
    for _ in range(3):  # several blocks per frame, so a frame's blocks can land on both sides of the cut
        blks = [W.valid_block(rnd, "text") for _ in range(4)]
        frames.append(W.frame([b for b, _ in blks]))
        frames.append(W.frame([b for b, _ in blks], content=b"".join(o for _, o in blks)))
    frames += W.raw_block_frames(rnd)
    frames += [W.frame([b]) for b in W.bad_blocks(rnd)]
    rnd.shuffle(frames)
    segs = [W.segment(frames[i::2]) for i in range(2)]
    kw = dict(synth.C2, lz4_linked_ppm=200000, lz4_content_checksum_ppm=200000, lz4_block_checksum_ppm=50000)
    segs += [gen(None, 6 << 20, i, **kw) for i in range(2)]
    got, ref = run_both(eng, O, segs, flags=DFLAGS)
    ok = (ref.batches["flags"] & abi.F_CODEC_OK) != 0
    assert int(np.sum(ok)) > len(frames) // 2
    assert_same(got, ref, DFLAGS)
    print(f"small_frec ok: {len(got.batches)} batches, {int(np.sum(ok))} decoded")


def case_zstd_ring_wave():
    """RPGPU_ZS_FAST=0: every zstd member through the wave decoder (ZDev, no
    lane parser), so the ring-mode members it turns down reach k_zexact from
    k_members_first rather than from k_zfallback; libzstd's bytes either way."""
    import random
    from oracle import oracle as O
    from redpanda_amd.engine import Engine
    from tests import zstd_corpus as ZC
    from tests.test_gpu_parity import _zstd_batches, assert_same, run_both
    assert os.environ.get("RPGPU_ZS_FAST") == "0"
    O.build()
    eng = Engine(0)
    rng = random.Random(7)
    frames = ZC.ring_frames(rng, 80)
    pay = [f for _, f in frames] + ZC.mutations(rng, frames[:10], per=3)
    got, ref = run_both(eng, O, [_zstd_batches(pay, counts=[1] * len(pay))], flags=DFLAGS)
    ok = (ref.batches["flags"] & abi.F_CODEC_OK) != 0
    assert int(np.sum(ok)) >= 40, int(np.sum(ok))
    assert_same(got, ref, DFLAGS)
    print(f"zstd_ring_wave ok: {len(got.batches)} batches, {int(np.sum(ok))} decoded")


CASES = {"small_pool": case_small_pool, "host_codec_missing": case_host_codec_missing, "small_frec": case_small_frec,
         "zstd_ring_wave": case_zstd_ring_wave}

if __name__ == "__main__":
    CASES[sys.argv[1]]()
