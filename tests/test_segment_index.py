"""Segment sparse-index rebuild during recovery.

Reference: checksumming_consumer::consume_batch_end -> segment_index::maybe_track
(storage/log_replayer.cc:62-74, storage/segment_index.cc:58-72) ->
index_state::maybe_index (storage/index_state.cc:48-95).

CPU tests pin the oracle (oracle/rp_oracle.c: rpo_segment_index) against the
reference's own test vectors (storage/tests/offset_index_utils_tests.cc) and a
small pure-Python restatement; GPU tests compare rpgpu_segment_index (one wave
per segment, rp_index.hip) with the oracle bit-exactly on the same job results.
"""
import numpy as np
import pytest

from redpanda_amd import abi
import synth  # noqa: E402  (test/bench data generator, not the product)

STEP = abi.INDEX_DEFAULT_STEP


def make_results(sizes, offsets, positions=None, first_ts=None, max_ts=None, lod=None, segs=None):
    """Synthetic rpgpu_batch_result rows + one summary per segment (all good)."""
    n = len(sizes)
    b = np.zeros(n, dtype=abi.BATCH_RESULT)
    b["size_bytes"] = sizes
    b["base_offset"] = offsets
    b["file_pos"] = positions if positions is not None else np.concatenate([[0], np.cumsum(sizes)[:-1]])
    b["first_timestamp"] = first_ts if first_ts is not None else 0
    b["max_timestamp"] = max_ts if max_ts is not None else 0
    b["last_offset_delta"] = lod if lod is not None else 0
    segs = segs or [(0, n, n)]
    sm = np.zeros(len(segs), dtype=abi.SEGMENT_SUMMARY)
    for k, (first, cnt, bad) in enumerate(segs):
        sm[k]["first_batch"] = first
        sm[k]["n_batches"] = cnt
        sm[k]["first_bad"] = bad
    return b, sm


def py_maybe_track(batches, sm, base_offset, step):
    """Pure-Python restatement of segment_index::maybe_track/index_state::maybe_index
    (storage/segment_index.cc:58-72, storage/index_state.cc:48-95)."""
    st = dict(base_offset=base_offset, max_offset=0, base_timestamp=0, max_timestamp=0, assert_batch=-1)
    ro, rt, ps = [], [], []
    acc = 0
    first = int(sm["first_batch"])
    for i in range(int(sm["first_bad"])):
        b = batches[first + i]
        if int(b["base_offset"]) < base_offset:
            st["assert_batch"] = i
            break
        acc += int(b["size_bytes"])
        retval = False
        if not ro:
            st["base_timestamp"] = st["max_timestamp"] = int(b["first_timestamp"])
            retval = True
        st["max_offset"] = int(b["base_offset"]) + int(b["last_offset_delta"])
        last_ts = max(int(b["first_timestamp"]), int(b["max_timestamp"]))
        st["max_timestamp"] = max(st["max_timestamp"], last_ts)
        if acc >= step or retval:
            ro.append((int(b["base_offset"]) - base_offset) & 0xFFFFFFFF)
            rt.append((last_ts - st["base_timestamp"]) & 0xFFFFFFFF)
            ps.append(int(b["file_pos"]))
            acc = 0
    return st, ro, rt, ps


def check_against_py(res, batches, summaries, bases, step):
    for k, (st, ro, rt, ps) in enumerate(res):
        pst, pro, prt, pps = py_maybe_track(batches, summaries[k], bases[k], step)
        for f in ("base_offset", "max_offset", "base_timestamp", "max_timestamp", "assert_batch"):
            assert int(st[f]) == pst[f], f
        assert list(ro) == pro and list(rt) == prt and list(ps) == pps


def find_nearest(st, ro, ps, o):
    """segment_index::find_nearest(offset) over the rebuilt entries
    (storage/segment_index.cc:89-107): the last entry at or below o."""
    if o < st["base_offset"] or len(ro) == 0:
        return None
    i = int(np.searchsorted(ro, np.uint32(o - int(st["base_offset"])), side="right")) - 1
    if i < 0:
        return None
    return int(st["base_offset"]) + int(ro[i]), int(ps[i])


# --- oracle pinned by the reference's own tests ------------------------------

def test_oracle_reference_vectors(oracle):
    """storage/tests/offset_index_utils_tests.cc:71-98 (index_truncate/bucket_truncate
    prologue): five batches indexed at their positions, the sixth (1667 B) not."""
    offs = [824, 849, 879, 901, 926, 948]
    sizes = [155103, 168865, 134080, 142073, 126886, 1667]
    pos = [0, 155103, 323968, 458048, 600121, 727007]
    b, sm = make_results(sizes, offs, positions=pos)
    (st, ro, rt, ps), = oracle.segment_index(b, sm, [0])
    assert list(ro) == [824, 849, 879, 901, 926]
    assert list(ps) == [0, 155103, 323968, 458048, 600121]
    assert find_nearest(st, ro, ps, 947) == (926, 600121)
    assert int(st["n_entries"]) == 5 and int(st["tracked"]) == 6


def test_oracle_round_trip_vector(oracle):
    """offset_index_utils_tests.cc:51-69 (index_round_trip): 1024 batches of
    default_data_buffer_step bytes -> 1024 entries, max_offset 1023."""
    n = 1024
    b, sm = make_results([STEP] * n, list(range(n)), positions=list(range(n)))
    (st, ro, rt, ps), = oracle.segment_index(b, sm, [0])
    assert int(st["max_offset"]) == 1023
    assert len(ro) == 1024 and list(ro) == list(range(n))


@pytest.mark.parametrize("seed", range(6))
def test_oracle_matches_python_restatement(oracle, seed):
    rng = np.random.default_rng(seed)
    nseg = 3
    counts = rng.integers(0, 400, nseg)
    n = int(counts.sum())
    sizes = np.exp(rng.uniform(np.log(61), np.log(200000), n)).astype(np.int64)
    offs = np.cumsum(rng.integers(1, 50, n))
    ts = 1_600_000_000_000 + np.cumsum(rng.integers(-5, 1000, n))
    mts = ts + rng.integers(-20, 500, n)
    segs, first = [], 0
    for c in counts:
        bad = int(rng.integers(0, c + 1)) if seed % 2 else int(c)
        segs.append((first, int(c), bad))
        first += int(c)
    b, sm = make_results(sizes, offs, first_ts=ts, max_ts=mts, lod=rng.integers(0, 20, n), segs=segs)
    step = [STEP, 0, 1, 4096, 1 << 20, STEP][seed]
    # base offsets: the first batch's offset, or one above it mid-segment (vassert path)
    bases = []
    for (f, c, _), k in zip(segs, range(nseg)):
        bases.append(int(offs[f + c // 2]) if (seed == 3 and c) else (int(offs[f]) if c else 0))
    res = oracle.segment_index(b, sm, bases, step=step)
    check_against_py(res, b, sm, bases, step)


# --- GPU: rpgpu_segment_index against the oracle -----------------------------

def _device_result(engine, b, sm):
    import torch
    from redpanda_amd.engine import DeviceResult
    dev = torch.device("cuda", engine.device)
    u8 = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(dev)
    return DeviceResult(batches=u8(b), records=None, decoded=None, summaries=u8(sm), totals=None, bitmap=None,
                        n_segments=len(sm))


def assert_index_same(got, ref):
    assert len(got) == len(ref)
    for (gs, gro, grt, gps), (rs, rro, rrt, rps) in zip(got, ref):
        for f in abi.INDEX_STATE.names:
            assert int(gs[f]) == int(rs[f]), f
        np.testing.assert_array_equal(gro, rro)
        np.testing.assert_array_equal(grt, rrt)
        np.testing.assert_array_equal(gps, rps)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_synthetic_results(engine, oracle, seed):
    rng = np.random.default_rng(100 + seed)
    nseg = 5
    counts = rng.integers(0, 3000, nseg)
    counts[0] = [0, 1, 63, 64, 65, 129][seed]
    n = int(counts.sum())
    sizes = np.exp(rng.uniform(np.log(61), np.log(1 << 20), n)).astype(np.int64)
    if seed == 4:
        sizes[:] = 16384  # the alternating chain of the C1 workload
    offs = np.cumsum(rng.integers(1, 50, n))
    ts = 1_600_000_000_000 + np.cumsum(rng.integers(-5, 1000, n))
    mts = ts + rng.integers(-20, 500, n)
    segs, first = [], 0
    for c in counts:
        bad = int(rng.integers(0, c + 1)) if seed % 2 else int(c)
        segs.append((first, int(c), bad))
        first += int(c)
    b, sm = make_results(sizes, offs, first_ts=ts, max_ts=mts, lod=rng.integers(0, 20, n), segs=segs)
    step = [STEP, 0, 1, 4096, STEP, 1 << 20][seed]
    bases = [int(offs[f + c // 2]) if (seed == 5 and c) else (int(offs[f]) if c else 0) for f, c, _ in segs]
    ref = oracle.segment_index(b, sm, bases, step=step)
    out = _device_result(engine, b, sm)
    got = engine.index_to_host(*engine.segment_index(out, bases, step=step), n_segments=nseg)
    assert_index_same(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["uniform16k", "tiny", "loguniform", "step0", "mixed_bad"])
def test_gpu_many_pieces(engine, oracle, kind):
    """Segments spanning many 1024-batch pieces: two candidates per piece
    (16 KiB batches), first entries past the 64 precomputed candidates (tiny
    batches: the serial fallback), log-uniform sizes, step 0, bad prefixes."""
    rng = np.random.default_rng(hash(kind) & 0xFFFF)
    counts = [20000, 1, 0, 4097, 9000]
    n = sum(counts)
    if kind in ("uniform16k", "step0"):
        sizes = np.full(n, 16384)
    elif kind == "tiny":
        sizes = rng.integers(61, 600, n)
    else:
        sizes = np.exp(rng.uniform(np.log(61), np.log(1 << 20), n)).astype(np.int64)
    offs = np.cumsum(rng.integers(1, 5, n))
    ts = 1_600_000_000_000 + np.cumsum(rng.integers(-5, 1000, n))
    segs, first = [], 0
    for c in counts:
        bad = int(rng.integers(0, c + 1)) if kind == "mixed_bad" else c
        segs.append((first, c, bad))
        first += c
    b, sm = make_results(sizes, offs, first_ts=ts, max_ts=ts + 7, lod=rng.integers(0, 3, n), segs=segs)
    step = 0 if kind == "step0" else STEP
    bases = [int(offs[f]) if c else 0 for f, c, _ in segs]
    if kind == "mixed_bad":
        bases[3] = int(offs[segs[3][0] + 3000])  # vassert mid-segment
    ref = oracle.segment_index(b, sm, bases, step=step)
    out = _device_result(engine, b, sm)
    got = engine.index_to_host(*engine.segment_index(out, bases, step=step), n_segments=len(counts))
    assert_index_same(got, ref)


@pytest.mark.gpu
def test_gpu_many_segments(engine, oracle):
    """Thousands of small segments (recovery of a long log): pieces are laid
    out densely (workspace ~ capacity / 1024 + segments, not their product),
    and the layout's scan crosses several 1024-segment rounds."""
    rng = np.random.default_rng(77)
    nseg = 3000
    counts = rng.integers(0, 40, nseg)
    counts[5] = 2500  # one segment of three pieces among them
    n = int(counts.sum())
    sizes = np.exp(rng.uniform(np.log(61), np.log(1 << 17), n)).astype(np.int64)
    offs = np.cumsum(rng.integers(1, 5, n))
    ts = 1_600_000_000_000 + np.cumsum(rng.integers(-5, 1000, n))
    segs, first = [], 0
    for c in counts:
        c = int(c)
        segs.append((first, c, int(rng.integers(0, c + 1)) if c and rng.random() < 0.3 else c))
        first += c
    b, sm = make_results(sizes, offs, first_ts=ts, max_ts=ts + 3, lod=rng.integers(0, 3, n), segs=segs)
    bases = [int(offs[f]) if c else 0 for f, c, _ in segs]
    ref = oracle.segment_index(b, sm, bases)
    out = _device_result(engine, b, sm)
    got = engine.index_to_host(*engine.segment_index(out, bases), n_segments=nseg)
    assert_index_same(got, ref)


@pytest.mark.gpu
def test_gpu_reference_vectors(engine, oracle):
    """offset_index_utils_tests.cc:71-98 and :51-69 through the device kernel."""
    offs = [824, 849, 879, 901, 926, 948] + list(range(2000, 3024))
    sizes = [155103, 168865, 134080, 142073, 126886, 1667] + [STEP] * 1024
    pos = [0, 155103, 323968, 458048, 600121, 727007] + list(range(1024))
    b, sm = make_results(sizes, offs, positions=pos, segs=[(0, 6, 6), (6, 1024, 1024)])
    out = _device_result(engine, b, sm)
    got = engine.index_to_host(*engine.segment_index(out, [0, 2000]), n_segments=2)
    (st, ro, rt, ps), (st2, ro2, _, _) = got
    assert list(ro) == [824, 849, 879, 901, 926] and list(ps) == [0, 155103, 323968, 458048, 600121]
    assert find_nearest(st, ro, ps, 947) == (926, 600121)
    assert int(st2["max_offset"]) == 3023 and list(ro2) == list(range(1024))
    assert_index_same(got, oracle.segment_index(b, sm, [0, 2000]))


@pytest.mark.gpu
def test_gpu_after_recovery_job(engine, oracle, rplib):
    """Real segments with corruption (the crc-good prefix is what gets tracked):
    engine job -> rpgpu_segment_index vs the oracle's job -> rpo_segment_index."""
    import torch
    segs = []
    for i in range(4):
        a = np.zeros(3 << 20, dtype=np.uint8)
        synth.gen_segment(a, i, seed=11 + i, batch_bytes=0, min_batch=200, max_batch=200000,
                          corrupt_payload_ppm=(20000 if i % 2 else 0), base_offset=1000 * i)
        segs.append(a)
    offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
    data = np.concatenate(segs)
    flags = abi.JOB_CRC | abi.JOB_PARSE
    ref_job = oracle.run_job(data, offs, flags)
    d = torch.from_numpy(data).cuda()
    nb = len(ref_job.batches)
    out = engine.alloc_outputs(len(segs), nb + 16, int(ref_job.totals["n_records"]) + 16, 1)
    engine.submit(d, offs, out, flags)
    bases = [1000 * i for i in range(len(segs))]
    got = engine.index_to_host(*engine.segment_index(out, bases), n_segments=len(segs))
    ref = oracle.segment_index(ref_job.batches, ref_job.summaries, bases, batch_cap=nb + 16)
    assert_index_same(got, ref)
    assert any(int(s["first_bad"]) < int(s["n_batches"]) for s in ref_job.summaries)  # the reject path ran
