#!/usr/bin/env python3
"""Benchmark: validated batch GB/s on device-resident Redpanda segments.

Workload (BASELINE.json configs[1] / [3]): per GPU, 8 partitions x one 2 GiB
on-disk segment of uncompressed 16 KiB record batches (seeded mt19937_64,
reference recipe), i.e. 16 GiB = 1,048,576 batches per GPU.  One step = the
whole pipeline over all 16 GiB: chain discovery, header_crc, batch CRC32C,
record walk into the offset index, log_replayer checkpoint, validity bitmap.
With --gpus N (torchrun, one rank per GPU) partitions are sharded p -> p % N
and the only collective is the final RCCL gather of bitmaps + segment
summaries to rank 0 (weak scaling).

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEG_BYTES = 2 << 30
PARTITIONS_PER_GPU = 8
BATCH_BYTES = 16384
SEED = 0xC1
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def gen_partitions(partitions, seg_bytes, batch_bytes, torch, device, threads=8):
    """Generate each partition's segment on the host (parallel, GIL released
    inside librpgpu) and copy it into one device buffer."""
    from redpanda_amd import _lib
    n = len(partitions)
    data = torch.empty(n * seg_bytes, dtype=torch.uint8, device=device)
    counts = [0] * n
    host_first = None
    lock = threading.Lock()
    sem = threading.Semaphore(threads)

    def work(i, p):
        nonlocal host_first
        with sem:
            buf = np.empty(seg_bytes, dtype=np.uint8)
            counts[i] = _lib.gen_segment(buf, p, seed=SEED, batch_bytes=batch_bytes)
            with lock:
                data[i * seg_bytes:(i + 1) * seg_bytes].copy_(torch.from_numpy(buf), non_blocking=False)
                if i == 0:
                    host_first = buf
    ths = [threading.Thread(target=work, args=(i, p)) for i, p in enumerate(partitions)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(seg_bytes)
    return data, offs, counts, host_first


def cpu_baseline(host_seg, seconds_budget=15.0):
    """The oracle's CPU restatement (SSE4.2 crc32c + record walk), timed on
    this box's host cores over a bounded sample of the same workload."""
    from oracle import oracle as O
    cores = min(16, os.cpu_count() or 1)
    sample = host_seg[: 1 << 30]  # 1 GiB sample = 65,536 batches
    # split the sample into `cores` slices on batch boundaries (16 KiB grid)
    per = (sample.size // BATCH_BYTES) // cores * BATCH_BYTES
    offs = np.arange(cores + 1, dtype=np.uint64) * np.uint64(per)
    sample = np.ascontiguousarray(sample[: int(offs[-1])])
    # 1 core, single slice (sanity of the per-core rate)
    one = np.ascontiguousarray(sample[:per])
    nb1, s1, b1 = O.baseline_validate(one, [0, per], 1)
    reps, total_b, total_s = 0, 0, 0.0
    while total_s < seconds_budget and reps < 20:
        nb, s, b = O.baseline_validate(sample, offs, cores)
        total_b += b
        total_s += s
        reps += 1
    return {
        "value": round(total_b / total_s / 1e9, 3),
        "unit": "GB/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{sample.size >> 20} MiB of the C1 workload (65,536-batch slice of partition 0), "
                  f"header_crc + batch CRC32C (SSE4.2) + record walk, {cores} threads x {reps} reps; "
                  f"1 core: {b1 / s1 / 1e9:.2f} GB/s",
        "one_core_GBs": round(b1 / s1 / 1e9, 3),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seg-gib", type=float, default=SEG_BYTES / (1 << 30))
    ap.add_argument("--partitions", type=int, default=PARTITIONS_PER_GPU)
    ap.add_argument("--chunk-kib", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", choices=["bitmap", "index"], default="bitmap")
    ap.add_argument("--no-parse", action="store_true", help="CRC only (diagnostic; not the headline workload)")
    ap.add_argument("--no-index", action="store_true", help="skip the segment-index rebuild measurement")
    ap.add_argument("--batch-bytes", type=int, default=BATCH_BYTES,
                    help="size_bytes per batch (diagnostic; the headline workload is 16 KiB)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from redpanda_amd import abi
    from redpanda_amd.engine import Engine
    from redpanda_amd.shard import as_bytes, gather_bytes, gather_job_verdicts, partitions_for_rank

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    seg_bytes = int(args.seg_gib * (1 << 30)) // BATCH_BYTES * BATCH_BYTES
    parts = partitions_for_rank(args.partitions * world, world, rank)
    t0 = time.time()
    data, offs, counts, host_first = gen_partitions(parts, seg_bytes, args.batch_bytes, torch, device)
    n_batches = int(sum(counts))
    log(f"[rank {rank}] generated {len(parts)} x {seg_bytes >> 20} MiB, {n_batches} batches in {time.time() - t0:.1f}s")

    eng = Engine(local)
    flags = abi.JOB_CRC | (0 if args.no_parse else abi.JOB_PARSE)
    rec_per_batch = 32
    out = eng.alloc_outputs(len(parts), n_batches + 16, n_batches * rec_per_batch, 1)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(device)
    chunk = args.chunk_kib << 10

    def step():
        eng.submit(data, offs, out, flags, chunk, d_seg_offsets=d_offs)
        if world > 1:
            # the one exchange: validity bitmaps + segment summaries to rank 0
            payload = [out.bitmap, out.summaries]
            if args.gather == "index":
                payload.append(out.batches)
            for t in payload:
                gather_bytes(as_bytes(t), rank, world, dist)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    # correctness of the measured workload (size-independent properties)
    h = out.to_host()
    nb = len(h.batches)
    all_ok = bool(nb == n_batches and (args.no_parse or np.all(h.batches["flags"] & abi.F_PARSE_OK))
                  and np.all(h.batches["flags"] & abi.F_CRC_OK) and h.totals["overflow"] == 0)
    bm_ok = bool(np.all(h.bitmap[: nb // 64] == np.uint64(0xFFFFFFFFFFFFFFFF)))
    n_records = int(h.totals["n_records"])
    if world > 1:
        # the gathered job picture on rank 0: every partition checkpointed at its end
        g = gather_job_verdicts(out.summaries, out.bitmap, nb, parts, rank, world, dist)
        if rank == 0:
            all_ok = bool(all_ok and np.all(g["summaries"]["has_checkpoint"] == 1)
                          and np.all(g["summaries"]["first_bad"] == g["summaries"]["n_batches"]))
    payload_bytes = int(np.sum(h.batches["size_bytes"].astype(np.int64) - abi.HEADER_SIZE))
    seg_total = int(np.sum(h.batches["size_bytes"].astype(np.int64)))
    del h

    eng.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    t2 = time.perf_counter()
    eng.set_timing(False)
    tm = eng.last_timings()
    elapsed = t2 - t1
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        tb = torch.tensor([seg_total, n_batches], dtype=torch.float64, device=device)
        dist.all_reduce(tb, op=dist.ReduceOp.SUM)
        job_bytes, job_batches = float(tb[0].item()), float(tb[1].item())
    else:
        job_bytes, job_batches = float(seg_total), float(n_batches)
    ms_per_step = elapsed / args.steps * 1e3
    value = job_bytes * args.steps / elapsed / 1e9

    # roofline of the dominant kernel (k_validate: CRC32C of every stored
    # payload): algorithmic bytes per launch = payload read once + 128 B per
    # batch result (descriptor read + verdict written, counted once).  The
    # record walk runs in k_walk (index writes: 64 B per record + the result
    # struct), reported beside it.
    alg = payload_bytes + 128 * n_batches
    v_ms = tm["validate"]
    achieved = alg / (v_ms * 1e-3) / 1e9
    walk_alg = 64 * n_records + 128 * n_batches
    w_ms = tm.get("walk", 0.0)
    traffic = None
    tfile = os.path.join(ROOT, "profiles", "validate_traffic.json")  # refreshed by scripts/parse_profile.py
    if os.path.exists(tfile):
        try:
            tj = json.load(open(tfile))
            # only a profile of the same kernel split counts
            if tj.get("alg_def") == "payload+128B/batch":
                traffic = tj.get("bytes_per_launch")
        except Exception:
            traffic = None

    # segment sparse-index rebuild (segment_index::maybe_track over the
    # recovered batches, §8(f) row 2): timed separately on its own stream,
    # after the headline region; not part of `value`
    index = None
    if not args.no_index:
        st = torch.cuda.Stream(device)
        bases = [0] * len(parts)
        torch.cuda.synchronize(device)
        with torch.cuda.stream(st):
            res = eng.segment_index(out, bases, stream=st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 5
            e0.record(st)
            for _ in range(reps):
                res = eng.segment_index(out, bases, stream=st, outputs=res)
            e1.record(st)
        st.synchronize()
        ix = eng.index_to_host(*res, n_segments=len(parts))
        n_entries = int(sum(int(r[0]["n_entries"]) for r in ix))
        gathered = None
        if world > 1:
            # the job's indexes at rank 0 (RCCL gather of the used entries only)
            from redpanda_amd.shard import gather_segment_index
            g = gather_segment_index(*res, parts, rank, world, dist)
            if rank == 0:
                gathered = {"partitions": len(g), "entries": int(sum(int(v[0]["n_entries"]) for v in g.values()))}
        index = {"kernel": "k_idx_cut+k_idx_cand+k_idx_resolve+k_idx_emit", "ms": round(e0.elapsed_time(e1) / reps, 4), "step": abi.INDEX_DEFAULT_STEP,
                 "entries": n_entries, "tracked": int(sum(int(r[0]["tracked"]) for r in ix)),
                 "gathered_at_rank0": gathered,
                 "note": "piece-parallel (1024-batch pieces, candidate first entries, serial resolve); "
                         "outputs preallocated, timed region = the four kernels + workspace memset"}
        del ix, res

    cpu = None
    if rank == 0 and not args.no_cpu_baseline and host_first is not None:
        cpu = cpu_baseline(host_first)
    if rank == 0:
        line = {
            "metric": "validated+decoded batch GB/s per GPU and whole node; % of HBM peak",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded mt19937_64, reference random_batch recipe), device-resident",
            "config": {
                "workload": "C1/C3: per GPU 8 partitions x 2 GiB disk segments of uncompressed 16 KiB batches "
                            "(seed 0xC1): chain discovery + header_crc + CRC32C + record walk/index + checkpoint",
                "segment_bytes": seg_bytes,
                "partitions_per_gpu": len(parts),
                "batches_per_gpu": n_batches,
                "records_per_gpu": n_records,
                "batch_bytes": args.batch_bytes,
                "batches_per_s": round(job_batches * args.steps / elapsed, 1),
                "parallelism": f"partition-sharded x{world}, RCCL gather of bitmaps+summaries",
                "parity": {"all_batches_valid": all_ok, "bitmap_all_ones": bm_ok},
                "stage_ms": {k: round(v, 4) for k, v in tm.items()},
                "hbm_fraction_whole_pipeline": round(value / world / HBM_PEAK_GBS, 4),
                "segment_index": index,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_validate",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "alg_bytes_per_launch": alg,
                "kernel_ms": round(v_ms, 4),
                "walk": {"kernel": "k_walk", "kernel_ms": round(w_ms, 4), "alg_bytes_per_launch": walk_alg,
                         "achieved": round(walk_alg / (w_ms * 1e-3) / 1e9, 1) if w_ms > 0 else None},
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
