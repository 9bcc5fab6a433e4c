"""Multi-GPU sharding of a recovery / validation job.

Partitions are independent: partition p is owned by rank p % world (the
reference's shard-per-core ownership, cluster/partition_manager, lifted to
one process per GPU).  Each rank validates its own segments with no
data-path collective; the one exchange is a gather of the per-segment
summaries (checkpoints) and validity bitmaps to rank 0, where a caller such
as log recovery wants the whole job's picture.

Everything here takes `dist` (torch.distributed) and works with the nccl
(RCCL) backend on device tensors and with gloo on host tensors; under gloo a
device payload is staged through host memory (gloo's gather has no device
path), which lets several ranks rehearse the N > 1 path on one card.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np


def partitions_for_rank(n_partitions: int, world: int, rank: int) -> List[int]:
    """Global partition ids owned by `rank` (p % world == rank)."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    return [p for p in range(n_partitions) if p % world == rank]


def _comm(t, dist):
    """`t` where the backend moves it: device tensors for nccl, host tensors
    for gloo."""
    if t.is_cuda and dist.get_backend() == "gloo":
        return t.cpu()
    return t


def gather_sizes(t, world: int, dist) -> List[int]:
    """Every rank's length of `t` (one small all_gather and a host sync):
    negotiate once, then pass the result to gather_bytes for repeated gathers
    of same-shaped payloads."""
    import torch
    n = _comm(torch.tensor([t.numel()], dtype=torch.int64, device=t.device), dist)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    return [int(s.item()) for s in sizes]


def gather_bytes(t, rank: int, world: int, dist, dst: int = 0, sizes: Sequence[int] = None):
    """Gather a 1-D uint8 tensor of any per-rank length to `dst`.  Returns the
    list of per-rank tensors on dst, None elsewhere.  The lengths come from
    `sizes` (gather_sizes) or one small all_gather; then one gather of
    equal-size (padded) buffers, with no host sync when `sizes` is given."""
    import torch
    if sizes is None:
        sizes = gather_sizes(t, world, dist)
    m = max(sizes) if sizes else 0
    t = _comm(t, dist)
    buf = t
    if t.numel() < m:
        buf = torch.zeros(m, dtype=t.dtype, device=t.device)
        buf[: t.numel()] = t
    if m == 0:
        return [t[:0] for _ in range(world)] if rank == dst else None
    if rank == dst:
        bufs = [torch.empty(m, dtype=t.dtype, device=t.device) for _ in range(world)]
        dist.gather(buf, bufs, dst=dst)
        return [b[:s] for b, s in zip(bufs, sizes)]
    dist.gather(buf, None, dst=dst)
    return None


def as_bytes(t):
    """View a contiguous tensor as flat uint8 (the gather payload)."""
    import torch
    return t.contiguous().view(torch.uint8).reshape(-1)


def gather_job_verdicts(summaries, bitmap, n_batches: int, parts: Sequence[int], rank: int, world: int, dist):
    """Gather each rank's segment summaries (rpgpu_segment_summary[len(parts)])
    and its validity bitmap (first n_batches bits) to rank 0.

    Returns on rank 0 a dict with `summaries`: a numpy structured array of
    all partitions in global partition order, and `bitmaps`: {partition
    rank's parts tuple: bits} per rank; None on other ranks."""
    import torch
    from . import abi
    meta = torch.tensor(list(parts) + [n_batches], dtype=torch.int64, device=summaries.device)
    got_meta = gather_bytes(as_bytes(meta), rank, world, dist)
    got_s = gather_bytes(as_bytes(summaries), rank, world, dist)
    got_b = gather_bytes(as_bytes(bitmap), rank, world, dist)
    if rank != 0:
        return None
    total = sum(len(m.cpu().numpy().view(np.int64)) - 1 for m in got_meta)
    out = np.zeros(total, dtype=abi.SEGMENT_SUMMARY)
    bits = {}
    for r in range(world):
        m = got_meta[r].cpu().numpy().view(np.int64)
        rp, nb = [int(x) for x in m[:-1]], int(m[-1])
        s = got_s[r].cpu().numpy().view(abi.SEGMENT_SUMMARY)
        if len(s) != len(rp):
            raise RuntimeError(f"rank {r}: {len(s)} summaries for {len(rp)} partitions")
        for i, p in enumerate(rp):
            out[p] = s[i]
        b = np.unpackbits(got_b[r].cpu().numpy(), bitorder="little")[:nb]
        bits[tuple(rp)] = b
    return {"summaries": out, "bitmaps": bits}


def gather_records(batches, records, summaries, parts: Sequence[int], rank: int, world: int, dist):
    """Gather each rank's per-batch results (rpgpu_batch_result[n_batches] as
    bytes) and per-record offset index (rpgpu_record_index[n_records] as
    bytes) to rank 0, and lay them out as ONE job over every partition in
    global partition order would have (the offset index at
    rank 0; what storage/log_replayer.cc:62-79 and the index rebuild need).

    On rank 0 the result is what a single-process job over all partitions
    (segment s = partition s) returns: batch `segment` = the partition id,
    batch ordinals and `index_base` continue across partitions, record
    `batch` = the global batch ordinal.  `decoded_off` stays rank-local (the
    decoded arena is not gathered).  None on other ranks."""
    import torch
    from . import abi
    meta = torch.tensor(list(parts), dtype=torch.int64, device=batches.device)
    got = [gather_bytes(as_bytes(t), rank, world, dist) for t in (meta, summaries[: len(parts) * abi.SEGMENT_SUMMARY.itemsize],
                                                               batches, records)]
    if rank != 0:
        return None
    per_part = {}
    for r in range(world):
        rp = got[0][r].cpu().numpy().view(np.int64)
        rs = got[1][r].cpu().numpy().view(abi.SEGMENT_SUMMARY)
        rb = got[2][r].cpu().numpy().view(abi.BATCH_RESULT)
        rr = got[3][r].cpu().numpy().view(abi.RECORD_INDEX)
        if len(rs) != len(rp):
            raise RuntimeError(f"rank {r}: {len(rs)} summaries for {len(rp)} partitions")
        rec0 = 0
        for p, s in zip(rp, rs):
            b0, nb, nrec = int(s["first_batch"]), int(s["n_batches"]), int(s["n_records"])
            if b0 + nb > len(rb) or rec0 + nrec > len(rr):
                raise RuntimeError(f"rank {r} partition {p}: results shorter than its summary")
            per_part[int(p)] = (rb[b0:b0 + nb], rr[rec0:rec0 + nrec], b0, rec0)
            rec0 += nrec
    bs, rs_ = [], []
    gb = gr = 0
    for p in sorted(per_part):
        b, rec, b0, r0 = per_part[p]
        b = b.copy()
        rec = rec.copy()
        b["segment"] = p
        # index_base: the record slot of the batch's first index entry
        b["index_base"] = b["index_base"] - np.uint64(r0) + np.uint64(gr)
        rec["batch"] = (rec["batch"].astype(np.int64) - b0 + gb).astype(np.uint32)
        bs.append(b)
        rs_.append(rec)
        gb += len(b)
        gr += len(rec)
    return {"batches": np.concatenate(bs) if bs else np.zeros(0, abi.BATCH_RESULT),
            "records": np.concatenate(rs_) if rs_ else np.zeros(0, abi.RECORD_INDEX),
            "partitions": sorted(per_part)}


def gather_segment_index(states, rel_off, rel_time, pos, parts: Sequence[int], rank: int, world: int, dist):
    """Gather each rank's rebuilt segment indexes (the outputs of
    Engine.segment_index: rpgpu_index_state[len(parts)] as bytes plus the three
    entry arrays) to rank 0.  Only the used entries travel: each rank packs
    segment s's entries [first_entry, first_entry + n_entries) back to back.

    Returns on rank 0 {partition: (index_state row, relative_offset,
    relative_time, position)} for every partition of the job; None elsewhere."""
    import torch
    from . import abi
    if states.is_cuda:
        # the index kernels may still run on the stream that produced them
        torch.cuda.synchronize(states.device)
    st = np.frombuffer(states.cpu().numpy().tobytes(), dtype=abi.INDEX_STATE)[: len(parts)]
    sl = [(int(s["first_entry"]), int(s["n_entries"])) for s in st]
    ro = torch.cat([rel_off[a:a + n] for a, n in sl]) if sl else rel_off[:0]
    rt = torch.cat([rel_time[a:a + n] for a, n in sl]) if sl else rel_time[:0]
    ps = torch.cat([pos[a:a + n] for a, n in sl]) if sl else pos[:0]
    meta = torch.tensor(list(parts), dtype=torch.int64, device=states.device)
    got = [gather_bytes(as_bytes(t), rank, world, dist) for t in (meta, states[: len(parts) * abi.INDEX_STATE.itemsize],
                                                                   ro, rt, ps)]
    if rank != 0:
        return None
    out = {}
    for r in range(world):
        rp = got[0][r].cpu().numpy().view(np.int64)
        rs = got[1][r].cpu().numpy().view(abi.INDEX_STATE)
        rro = got[2][r].cpu().numpy().view(np.uint32)
        rrt = got[3][r].cpu().numpy().view(np.uint32)
        rps = got[4][r].cpu().numpy().view(np.uint64)
        if len(rs) != len(rp):
            raise RuntimeError(f"rank {r}: {len(rs)} index states for {len(rp)} partitions")
        k = 0
        for p, s in zip(rp, rs):
            n = int(s["n_entries"])
            out[int(p)] = (s, rro[k:k + n], rrt[k:k + n], rps[k:k + n])
            k += n
    return out
