"""Multi-rank path (redpanda_amd/shard.py) with gloo, world_size 2, on CPU.

Each rank owns partitions p % world == rank and runs the oracle over them in
place of the device engine (this test covers sharding and the gather, not
the kernels); rank 0 must end with every partition's summary in global
order and each rank's validity bits, equal to a single-process run.
"""
import json
import os
import socket

import numpy as np
import pytest

from redpanda_amd import abi
from redpanda_amd.shard import partitions_for_rank
import synth  # noqa: E402  (test/bench data generator, not the product)

N_PARTS = 5
SEG = 300_000
KW = dict(seed=0xE5, batch_bytes=0, min_batch=300, max_batch=40_000, corrupt_payload_ppm=80_000)
SUMMARY_FIELDS = ["n_batches", "terminal_pos", "bytes_consumed", "terminal_errc", "terminal_eof", "has_checkpoint",
                  "first_bad", "ckpt_last_offset", "ckpt_truncate_pos", "n_records"]


def _segments(parts):
    from redpanda_amd import _lib
    segs = []
    for p in parts:
        a = np.zeros(SEG + 997 * p, dtype=np.uint8)  # ragged per-partition sizes
        synth.gen_segment(a, p, **KW)
        segs.append(a)
    return segs


def _oracle_job(segs):
    from oracle import oracle as O
    offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
    data = np.concatenate(segs) if segs else np.zeros(0, np.uint8)
    return O.run_job(data, offs, abi.JOB_CRC | abi.JOB_PARSE)


def _worker(rank, world, port, out_path):
    import torch
    import torch.distributed as dist
    from redpanda_amd.shard import gather_job_verdicts
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        parts = partitions_for_rank(N_PARTS, world, rank)
        res = _oracle_job(_segments(parts))
        summaries = torch.from_numpy(res.summaries.copy().view(np.uint8))
        bitmap = torch.from_numpy(res.bitmap.copy().view(np.uint8))
        got = gather_job_verdicts(summaries, bitmap, len(res.batches), parts, rank, world, dist)
        if rank == 0:
            s = got["summaries"]
            json.dump({"summaries": {f: s[f].tolist() for f in SUMMARY_FIELDS},
                       "bitmaps": {",".join(map(str, k)): v.tolist() for k, v in got["bitmaps"].items()}},
                      open(out_path, "w"))
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_partition_ownership():
    for world in (1, 2, 3, 8):
        owned = [partitions_for_rank(17, world, r) for r in range(world)]
        assert sorted(p for o in owned for p in o) == list(range(17))
        assert all(p % world == r for r, o in enumerate(owned) for p in o)
    with pytest.raises(ValueError):
        partitions_for_rank(4, 2, 2)


def test_gloo_world2_gather_matches_single_process(rplib, oracle, tmp_path):
    import torch.multiprocessing as mp
    out = str(tmp_path / "rank0.json")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = json.load(open(out))
    # single-process reference: every partition on its own
    for p in range(N_PARTS):
        ref = _oracle_job(_segments([p]))
        for f in SUMMARY_FIELDS:
            assert got["summaries"][f][p] == ref.summaries[f][0].item(), (p, f)
    assert any(v == 0 for b in got["bitmaps"].values() for v in b), "corruption should clear some bits"
    for r in range(2):
        parts = partitions_for_rank(N_PARTS, 2, r)
        want = np.concatenate([np.unpackbits(_oracle_job(_segments([p])).bitmap.view(np.uint8),
                                             bitorder="little")[: len(_oracle_job(_segments([p])).batches)]
                               for p in parts])
        assert got["bitmaps"][",".join(map(str, parts))] == want.tolist()


def _index_worker(rank, world, port, out_path):
    """Per rank: oracle job + oracle index rebuild over its partitions (in place
    of the device engine), then the gather of the indexes to rank 0."""
    import torch
    import torch.distributed as dist
    from oracle import oracle as O
    from redpanda_amd.shard import gather_segment_index
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        parts = partitions_for_rank(N_PARTS, world, rank)
        res = _oracle_job(_segments(parts))
        ix = O.segment_index(res.batches, res.summaries, [0] * len(parts), step=4096)
        cap = max(len(res.batches), 1)
        st = np.zeros(len(parts), dtype=abi.INDEX_STATE)
        ro, rt, ps = np.zeros(cap, np.uint32), np.zeros(cap, np.uint32), np.zeros(cap, np.uint64)
        for k, (s, a, b, c) in enumerate(ix):
            st[k] = s
            f, n = int(s["first_entry"]), int(s["n_entries"])
            ro[f:f + n], rt[f:f + n], ps[f:f + n] = a, b, c
        got = gather_segment_index(torch.from_numpy(st.view(np.uint8).copy()), torch.from_numpy(ro.view(np.int32)),
                                   torch.from_numpy(rt.view(np.int32)), torch.from_numpy(ps.view(np.int64)),
                                   parts, rank, world, dist)
        if rank == 0:
            json.dump({str(p): {"n": int(v[0]["n_entries"]), "max_offset": int(v[0]["max_offset"]),
                                "ro": v[1].tolist(), "ps": v[3].tolist()} for p, v in got.items()},
                      open(out_path, "w"))
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


def test_gloo_world2_index_gather_matches_single_process(rplib, oracle, tmp_path):
    import torch.multiprocessing as mp
    out = str(tmp_path / "rank0_index.json")
    mp.spawn(_index_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = json.load(open(out))
    assert sorted(int(p) for p in got) == list(range(N_PARTS))
    for p in range(N_PARTS):
        ref = _oracle_job(_segments([p]))
        (s, ro, rt, ps), = oracle.segment_index(ref.batches, ref.summaries, [0], step=4096)
        g = got[str(p)]
        assert g["n"] == int(s["n_entries"]) > 0 and g["max_offset"] == int(s["max_offset"])
        assert g["ro"] == ro.tolist() and g["ps"] == ps.tolist()


# ---------------------------------------------------------------------------
# The whole gather (verdicts, segment index, per-batch results and the
# per-record offset index) over per-rank job outputs saved as host arrays:
# by the oracle here, by the HIP engine on cuda:0 in the -m gpu test.  The
# gloo workers never touch the GPU; rank 0 must hold exactly what ONE
# single-process oracle job over every partition (global order) returns.
# ---------------------------------------------------------------------------
INDEX_STEP = 4096


def _save_rank(path, res, ix, parts):
    st = np.zeros(len(parts), dtype=abi.INDEX_STATE)
    cap = max(len(res.batches), 1)
    ro, rt, ps = np.zeros(cap, np.uint32), np.zeros(cap, np.uint32), np.zeros(cap, np.uint64)
    for k, (s, a, b, c) in enumerate(ix):
        st[k] = s
        f, n = int(s["first_entry"]), int(s["n_entries"])
        ro[f:f + n], rt[f:f + n], ps[f:f + n] = a, b, c
    np.savez(path, batches=res.batches.view(np.uint8), records=res.records.view(np.uint8),
             summaries=res.summaries.view(np.uint8), bitmap=res.bitmap.view(np.uint8), n_batches=len(res.batches),
             parts=np.asarray(parts, np.int64), states=st.view(np.uint8), ro=ro, rt=rt, ps=ps)


def _full_gather_worker(rank, world, port, in_dir, out_path):
    import torch
    import torch.distributed as dist
    from redpanda_amd.shard import gather_job_verdicts, gather_records, gather_segment_index
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        z = np.load(os.path.join(in_dir, f"rank{rank}.npz"))
        parts = [int(p) for p in z["parts"]]
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
        v = gather_job_verdicts(t(z["summaries"]), t(z["bitmap"]), int(z["n_batches"]), parts, rank, world, dist)
        ix = gather_segment_index(t(z["states"]), t(z["ro"].view(np.int32)), t(z["rt"].view(np.int32)),
                                  t(z["ps"].view(np.int64)), parts, rank, world, dist)
        rec = gather_records(t(z["batches"]), t(z["records"]), t(z["summaries"]), parts, rank, world, dist)
        if rank == 0:
            np.savez(out_path, summaries=v["summaries"].view(np.uint8),
                     bits=np.concatenate([v["bitmaps"][k] for k in sorted(v["bitmaps"])]),
                     batches=rec["batches"].view(np.uint8), records=rec["records"].view(np.uint8),
                     ix_n=np.asarray([int(ix[p][0]["n_entries"]) for p in range(N_PARTS)]),
                     ix_ro=np.concatenate([ix[p][1] for p in range(N_PARTS)]),
                     ix_ps=np.concatenate([ix[p][3] for p in range(N_PARTS)]))
        else:
            assert v is None and ix is None and rec is None
    finally:
        dist.destroy_process_group()


def _check_full_gather(out_path, oracle):
    import torch.multiprocessing as mp  # noqa: F401
    z = np.load(out_path)
    ref = _oracle_job(_segments(list(range(N_PARTS))))
    got_s = z["summaries"].view(abi.SEGMENT_SUMMARY)
    for f in SUMMARY_FIELDS:
        assert np.array_equal(got_s[f], ref.summaries[f]), f
    gb = z["batches"].view(abi.BATCH_RESULT)
    gr = z["records"].view(abi.RECORD_INDEX)
    assert len(gb) == len(ref.batches) > 0 and len(gr) == len(ref.records) > 0
    for f in abi.BATCH_COMPARE_FIELDS:
        if f != "decoded_off":
            assert np.array_equal(gb[f], ref.batches[f]), f"batches.{f}"
    for f in abi.RECORD_COMPARE_FIELDS:
        assert np.array_equal(gr[f], ref.records[f]), f"records.{f}"
    # per-rank bitmaps, rank order = sorted parts tuples
    assert not np.all(z["bits"] == 1), "corruption should clear some bits"
    ixr = oracle.segment_index(ref.batches, ref.summaries, [0] * N_PARTS, step=INDEX_STEP)
    assert z["ix_n"].tolist() == [int(s["n_entries"]) for s, _, _, _ in ixr]
    assert np.array_equal(z["ix_ro"], np.concatenate([r[1] for r in ixr]))
    assert np.array_equal(z["ix_ps"], np.concatenate([r[3] for r in ixr]))


def test_gloo_world2_full_gather_oracle_outputs(rplib, oracle, tmp_path):
    import torch.multiprocessing as mp
    for r in range(2):
        parts = partitions_for_rank(N_PARTS, 2, r)
        res = _oracle_job(_segments(parts))
        ix = oracle.segment_index(res.batches, res.summaries, [0] * len(parts), step=INDEX_STEP)
        _save_rank(str(tmp_path / f"rank{r}.npz"), res, ix, parts)
    out = str(tmp_path / "rank0_full.npz")
    mp.spawn(_full_gather_worker, args=(2, _free_port(), str(tmp_path), out), nprocs=2, join=True)
    _check_full_gather(out, oracle)


@pytest.mark.gpu
def test_gloo_world2_full_gather_gpu_outputs(rplib, oracle, tmp_path):
    """Config C3 in miniature: the HIP engine validates each rank's
    partitions on cuda:0 (records, summaries, bitmap, segment index), the
    CPU-only gloo ranks gather those outputs to rank 0."""
    import torch
    import torch.multiprocessing as mp
    from redpanda_amd.engine import Engine
    eng = Engine(0)
    for r in range(2):
        parts = partitions_for_rank(N_PARTS, 2, r)
        segs = _segments(parts)
        offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
        data = torch.from_numpy(np.concatenate(segs)).cuda()
        flags = abi.JOB_CRC | abi.JOB_PARSE
        total = int(offs[-1])
        out = eng.alloc_outputs(len(parts), total // abi.HEADER_SIZE + 16, total // 4, 1)
        eng.submit(data, offs, out, flags)
        torch.cuda.synchronize()
        res = out.to_host()
        ix = eng.index_to_host(*eng.segment_index(out, [0] * len(parts), step=INDEX_STEP), n_segments=len(parts))
        _save_rank(str(tmp_path / f"rank{r}.npz"), res, ix, parts)
    eng.close()
    out = str(tmp_path / "rank0_full.npz")
    mp.spawn(_full_gather_worker, args=(2, _free_port(), str(tmp_path), out), nprocs=2, join=True)
    _check_full_gather(out, oracle)


@pytest.mark.gpu
def test_rccl_world1_gather_device_tensors(rplib, oracle):
    """bench.py's nccl branch (RCCL) on one GPU: a 1-rank nccl process group
    opened with device_id, as `bench.py --gpus N` opens it, runs every gather
    of §8(e) (sizes, bytes, verdicts, batch results + record index, segment
    index) on the device tensors of a real HIP job; rank 0's picture must be
    the local job's and the oracle's (storage/log_replayer.cc:62-79)."""
    import torch
    import torch.distributed as dist
    from redpanda_amd.engine import Engine
    from redpanda_amd.shard import as_bytes, gather_bytes, gather_job_verdicts, gather_records, gather_segment_index, \
        gather_sizes
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    eng = Engine(0)
    parts = list(range(N_PARTS))
    segs = _segments(parts)
    offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
    data = torch.from_numpy(np.concatenate(segs)).to(dev)
    total = int(offs[-1])
    out = eng.alloc_outputs(len(parts), total // abi.HEADER_SIZE + 16, total // 4, 1)
    eng.submit(data, offs, out, abi.JOB_CRC | abi.JOB_PARSE)
    torch.cuda.synchronize()
    local = out.to_host()
    nb, nr = len(local.batches), len(local.records)
    ixo = eng.segment_index(out, [0] * len(parts), step=INDEX_STEP)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        bm = as_bytes(out.bitmap)
        sz = gather_sizes(bm, 1, dist)
        assert sz == [bm.numel()]
        g = gather_bytes(bm, 0, 1, dist, sizes=sz)
        assert g[0].is_cuda and torch.equal(g[0], bm)
        v = gather_job_verdicts(out.summaries, out.bitmap, nb, parts, 0, 1, dist)
        rec = gather_records(out.batches[: nb * abi.BATCH_RESULT.itemsize],
                             out.records[: nr * abi.RECORD_INDEX.itemsize], out.summaries, parts, 0, 1, dist)
        ix = gather_segment_index(*ixo, parts, 0, 1, dist)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    ref = _oracle_job(segs)
    for f in SUMMARY_FIELDS:
        assert np.array_equal(v["summaries"][f], ref.summaries[f]), f
        assert np.array_equal(v["summaries"][f], local.summaries[f]), f
    bits = np.unpackbits(ref.bitmap.view(np.uint8), bitorder="little")[: len(ref.batches)]
    assert np.array_equal(v["bitmaps"][tuple(parts)], bits) and not np.all(bits == 1)
    assert len(rec["batches"]) == len(ref.batches) > 0 and len(rec["records"]) == len(ref.records) > 0
    for f in abi.BATCH_COMPARE_FIELDS:
        if f != "decoded_off":
            assert np.array_equal(rec["batches"][f], ref.batches[f]), f"batches.{f}"
    for f in abi.RECORD_COMPARE_FIELDS:
        assert np.array_equal(rec["records"][f], ref.records[f]), f"records.{f}"
    ixr = oracle.segment_index(ref.batches, ref.summaries, [0] * N_PARTS, step=INDEX_STEP)
    for p, (s, ro, rt, ps) in enumerate(ixr):
        assert int(ix[p][0]["n_entries"]) == int(s["n_entries"]) > 0
        assert np.array_equal(ix[p][1], ro) and np.array_equal(ix[p][3], ps)
    eng.close()
