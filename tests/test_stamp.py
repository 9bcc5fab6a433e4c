"""Write side: header stamping of batches about to be
written — disk_log_appender::operator() (storage/disk_log_appender.cc:72-74,
:113-119: base_offset = the appender's next offset, header_crc) and
storage::internal::reset_size_checksum_metadata (storage/parser_utils.cc:
114-120: size_bytes, crc, header_crc).

The oracle (oracle/rp_oracle.c: rpo_stamp_batches) is pinned by segments
whose headers were written independently: the generator's appender
(synth/rp_gen.cpp) and the golden segments the reference's own Python reader
accepted (tests/golden, make_golden.py) — blanking the stamped fields and
stamping again must give back the same bytes.  The GPU (rpgpu_stamp) is
compared bit-exactly with the oracle, and a stamped job validates.
"""
import json
import os

import numpy as np
import pytest

from redpanda_amd import abi
import synth  # noqa: E402  (test/bench data generator, not the product)

HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")
OFFSETS, CRC = 1, 2


def blank(seg, pos, offsets=True, crc=True):
    z = seg.copy()
    for p in pos:
        p = int(p)
        z[p:p + 4] = 0  # header_crc
        if crc:
            z[p + 4:p + 8] = 0  # size_bytes
            z[p + 17:p + 21] = 0  # crc
        if offsets:
            z[p + 8:p + 16] = 0  # base_offset
    return z


def layout(oracle, seg):
    r = oracle.run_job(seg, [0, seg.size], abi.JOB_CRC)
    b = r.batches
    return b, b["file_pos"].astype(np.uint64), (b["size_bytes"] - abi.HEADER_SIZE).astype(np.uint32)


@pytest.mark.parametrize("recipe", ["c1", "c5_clean", "lz4"])
def test_oracle_restamps_generated_segments(oracle, recipe):
    a = np.zeros(4 << 20, dtype=np.uint8)
    kw = {"c1": dict(seed=0xC1),
          "c5_clean": dict(seed=0xC5, batch_bytes=0, min_batch=200, max_batch=300000, weights=[40, 0, 15, 30, 0, 15]),
          "lz4": dict(seed=0xC2, batch_bytes=0, min_batch=4096, max_batch=1 << 20, weights=[0, 0, 0, 1, 0, 0])}[recipe]
    synth.gen_segment(a, 3, **kw)
    b, pos, pl = layout(oracle, a)
    assert len(b) > 3 and np.all(b["flags"] & abi.F_CRC_OK)
    end = int(pos[-1]) + int(pl[-1]) + abi.HEADER_SIZE
    first = int(b["base_offset"][0])
    # the generator's appender numbers batches as disk_log_appender does
    np.testing.assert_array_equal(b["base_offset"][1:], b["base_offset"][:-1] + b["last_offset_delta"][:-1] + 1)
    for flags in (OFFSETS | CRC, CRC, OFFSETS):
        z = blank(a, pos, offsets=bool(flags & OFFSETS), crc=bool(flags & CRC))
        st = oracle.stamp_batches(z, pos, pl, first, flags)
        np.testing.assert_array_equal(st[:end], a[:end])


def test_oracle_restamps_golden_segments(oracle):
    """Segments the reference's Python reader accepted (make_golden.py)."""
    man = json.load(open(os.path.join(G, "manifest.json")))
    n = 0
    for ent in man["segments"]:
        seg = np.fromfile(os.path.join(G, "segments", ent["name"] + ".bin"), dtype=np.uint8)
        r = oracle.run_job(seg, [0, seg.size], abi.JOB_CRC)
        b = r.batches
        good = (b["flags"] & abi.F_CRC_OK) != 0
        if not np.any(good):
            continue
        pos = b["file_pos"][good].astype(np.uint64)
        pl = (b["size_bytes"][good] - abi.HEADER_SIZE).astype(np.uint32)
        z = blank(seg, pos, offsets=False)
        st = oracle.stamp_batches(z, pos, pl, 0, CRC)
        for p, ln in zip(pos, pl):
            p = int(p)
            np.testing.assert_array_equal(st[p:p + abi.HEADER_SIZE + int(ln)], seg[p:p + abi.HEADER_SIZE + int(ln)])
        n += 1
    assert n >= 5


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [OFFSETS | CRC, CRC, OFFSETS])
def test_gpu_stamp_matches_oracle(engine, oracle, rplib, flags):
    """rpgpu_stamp == rpo_stamp_batches bit for bit (headers with arbitrary
    stale fields, payloads 0 B .. 1 MiB, a negative last_offset_delta), and
    the stamped job validates on the GPU."""
    import torch
    rng = np.random.default_rng(flags)
    segs = []
    for i, kw in enumerate([dict(seed=0xC1), dict(seed=0xC5, batch_bytes=0, min_batch=61, max_batch=1 << 20,
                                                 weights=[40, 0, 15, 30, 0, 15])]):
        a = np.zeros(6 << 20, dtype=np.uint8)
        synth.gen_segment(a, i, **kw)
        segs.append(a)
    data = np.concatenate(segs)
    offs = np.array([0, segs[0].size, data.size], dtype=np.uint64)
    r = oracle.run_job(data, offs, abi.JOB_CRC)
    b = r.batches
    pos = (b["file_pos"] + offs[b["segment"]]).astype(np.uint64)
    pl = (b["size_bytes"] - abi.HEADER_SIZE).astype(np.uint32)
    stale = data.copy()
    for p in pos:
        p = int(p)
        stale[p:p + 21] = rng.integers(0, 256, 21, dtype=np.uint8)
        stale[p + 16] = data[p + 16]  # keep the type byte
    stale[int(pos[5]) + 23:int(pos[5]) + 27] = np.frombuffer(np.int32(-7).tobytes(), np.uint8)  # lod < 0
    want = oracle.stamp_batches(stale, pos, pl, 1 << 40, flags)
    d = torch.from_numpy(np.concatenate([stale, np.zeros(16, np.uint8)])).cuda()
    engine.stamp(d, pos, pl, 1 << 40, flags)
    got = d[: data.size].cpu().numpy()
    np.testing.assert_array_equal(got, want)
    if flags & CRC:
        res = engine.validate(d[: data.size], offs, abi.JOB_CRC | abi.JOB_PARSE)
        assert len(res.batches) == len(b)
        assert np.all(res.batches["flags"] & abi.F_CRC_OK) and np.all(res.batches["flags"] & abi.F_HEADER_OK)
