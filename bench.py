#!/usr/bin/env python3
"""Benchmark: validated (+decoded) batch GB/s on device-resident Redpanda
segments, with the roofline of the dominant kernel and the CPU baseline.

Headline workload (BASELINE.json configs[1] / [3], `value`): per GPU, 8
partitions x one 2 GiB on-disk segment of uncompressed 16 KiB record batches
(seeded mt19937_64, reference recipe), i.e. 16 GiB = 1,048,576 batches per
GPU.  One step = the whole pipeline over all 16 GiB: chain discovery,
header_crc, batch CRC32C, record walk into the offset index, log_replayer
checkpoint, validity bitmap.  With --gpus N (torchrun, one rank per GPU)
partitions are sharded p -> p % N and the only collective is the final RCCL
gather of bitmaps + segment summaries to rank 0 (weak scaling).

At N = 1 three more stanzas ride on the same JSON line (configs[2] and [4],
SURVEY.md §8(d)): `c2` (LZ4 frames, 64 KiB..1 MiB decoded batches, decode +
CRC + parse), `c5` (skewed 200 B..1 MiB, none/lz4/snappy-java/raw snappy,
corruptions) and `c6` (C5 plus gzip / zstd), each with its own decode-stage
roofline and a CPU baseline over the reference's codec libraries.

Prints ONE JSON line on rank 0 (contract in the task statement).  Only the
headline's own timed region can cost that line: every stanza, baseline,
index measurement and gather check reports its failure inside its own field.

The device layer is `CudaPlatform` (torch-ROCm); tests/test_bench.py runs
this file's whole control flow (every stanza, and the N > 1 gather with gloo
at world size 2) on the CPU through a stand-in platform.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import synth  # noqa: E402  (test/bench data generator, not the product)

SEG_BYTES = 2 << 30
PARTITIONS_PER_GPU = 8
BATCH_BYTES = 16384
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# C2: 8 partitions x 1.5 GiB of LZ4 segments (~16 GiB decoded per GPU);
# C5 / C6: 128 partitions x 64 MiB (skewed batches, corruptions end chains early)
C2_PARTS, C2_SEG = 8, 3 << 29
C5_PARTS, C5_SEG = 128, 64 << 20
# C6's CPU sample: the first C6_CPU_PARTS partitions (1 MiB gzip / zstd
# batches take the reference's loops milliseconds each)
C6_CPU_PARTS = 8
CPU_C1_SAMPLE = 1 << 30
# rpgpu_validate_host's staging group (group_kib 0): whole segments up to 256 MiB
HOST_GROUP_BYTES = 256 << 20

# index writes 48 B per record, result 64 B per batch
IDX_BYTES_PER_RECORD = 48
RESULT_BYTES_PER_BATCH = 64
# (since round 6 the decode stage also holds k_crc_compose, the side-stream
# content checksums and k_dchain, which ran in the validate stage before)
DECODE_KERNELS = ("k_decode", "k_decode_blocks", "k_lzf_walk", "k_lzf_tail", "k_raw_copy", "k_lz_walk", "k_lz_exec",
                  "k_decode_finish", "k_crc_compose", "k_content_xxh", "k_dchain", "k_content_apply")
MEMBER_KERNELS = ("k_gzsplan", "k_gzsfind", "k_gzsdecode", "k_gzsresolve", "k_members_first", "k_zplan", "k_zlits",
                  "k_zparse", "k_zfallback", "k_zexec", "k_members", "k_inflate_copy")
# segment-summary fields that do not depend on where a partition sits in a job
SUMMARY_JOB_FIELDS = ("n_batches", "terminal_pos", "bytes_consumed", "terminal_errc", "terminal_eof",
                      "has_checkpoint", "first_bad", "ckpt_last_offset", "ckpt_truncate_pos", "n_records")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def failure(where, e):
    """A stanza / leg that failed: logged in full, reported in its field."""
    log(f"[{where}] failed: {e!r}\n{traceback.format_exc()}")
    return {"error": repr(e)}


class CudaPlatform:
    """The device layer the bench drives: torch-ROCm on an MI355X, one rank
    per GPU (LOCAL_RANK modulo the visible devices, so several ranks may
    share one card for a rehearsal of the N > 1 path)."""

    def __init__(self, local: int):
        import torch
        self.torch = torch
        n = torch.cuda.device_count()
        self.device = torch.device("cuda", local % max(n, 1))
        torch.cuda.set_device(self.device)

    def engine(self):
        from redpanda_amd.engine import Engine
        return Engine(self.device.index)

    def sync(self):
        self.torch.cuda.synchronize(self.device)

    def empty_cache(self):
        self.torch.cuda.empty_cache()

    def comm_device(self, backend: str):
        """Where collective tensors live: device memory for nccl (RCCL), the
        host for gloo."""
        return self.device if backend == "nccl" else self.torch.device("cpu")

    def host_segments(self, data, seg_bytes: int, n: int):
        """The job's n segments copied back into pinned host memory (the
        host-resident input of the H2D stanza)."""
        torch = self.torch
        out = []
        for i in range(n):
            t = torch.empty(seg_bytes, dtype=torch.uint8, pin_memory=True)
            t.copy_(data[i * seg_bytes:(i + 1) * seg_bytes])
            out.append(t.numpy())
        return out

    def time_on_side_stream(self, first, again, reps: int):
        """first(stream) once untimed, then `reps` x again(stream, prev)
        between HIP events recorded on that stream: (ms per call, result)."""
        torch = self.torch
        st = torch.cuda.Stream(self.device)
        self.sync()
        with torch.cuda.stream(st):
            res = first(st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(reps):
                res = again(st, res)
            e1.record(st)
        st.synchronize()
        return e0.elapsed_time(e1) / reps, res


def profiled_traffic(fname, workload, kernels):
    """HBM bytes per launch from the committed PMC summary
    (scripts/parse_traffic.py -> profiles/<fname>): the sum over `kernels`
    and the per-kernel table (bytes, algorithmic bytes, ratio)."""
    path = os.path.join(ROOT, "profiles", fname)
    try:
        with open(path) as f:
            tj = json.load(f).get(workload)
    except Exception:
        return None, None
    if not tj:
        return None, None
    ks = tj.get("kernels", {})
    tot = [ks[k]["bytes"] for k in kernels if k in ks and ks[k].get("bytes") is not None]
    return (int(sum(tot)) if tot else None), {"source": f"profiles/{fname} ({tj.get('tag')})", **ks}


def write_stats(args, name, d):
    """Merge one workload's byte counts into --stats-out (per-kernel
    algorithmic bytes for the PMC summary, scripts/parse_traffic.py)."""
    if not args.stats_out:
        return
    try:
        with open(args.stats_out) as f:
            cur = json.load(f)
    except Exception:
        cur = {}
    cur[name] = d
    with open(args.stats_out, "w") as f:
        json.dump(cur, f, indent=1)


def _lz4_seq_count(blk: bytes) -> int:
    """Sequences of one LZ4 block (token walk; the last literal run counts)."""
    ip, n, k = 0, len(blk), 0
    while ip < n:
        t = blk[ip]
        ip += 1
        ll = t >> 4
        if ll == 15:
            while ip < n:
                x = blk[ip]
                ip += 1
                ll += x
                if x != 255:
                    break
        ip += ll
        k += 1
        if ip + 2 > n:
            break
        ip += 2
        if (t & 15) == 15:
            while ip < n:
                x = blk[ip]
                ip += 1
                if x != 255:
                    break
    return k


def lz4_composition(seg: np.ndarray, file_pos, sizes, attrs, decoded_len=None, seq_sample: int = 300):
    """Byte composition of one segment's LZ4F payloads for the per-kernel
    algorithmic bytes (scripts/parse_traffic.py): stored (raw) block bytes
    (k_raw_copy's), compressed block bytes and the sequences they parse into
    (k_lzf_walk's / k_lz_exec's; sequences counted on the first seq_sample
    compressed blocks and scaled by compressed bytes).  Frame headers only,
    no decoding."""
    import struct
    raw = comp = nblk = lz4_out = 0
    sampled_bytes = sampled_seq = 0
    if decoded_len is None:
        decoded_len = np.zeros(len(sizes), np.int64)
    for pos, size, a, dl in zip(file_pos, sizes, attrs, decoded_len):
        if (int(a) & 7) != 3:
            continue
        lz4_out += int(dl)
        pay = seg[int(pos) + 61:int(pos) + int(size)].tobytes()
        if len(pay) < 7 or pay[:4] != b"\x04\x22\x4d\x18":
            continue
        flg = pay[4]
        p = 7 + (8 if flg & 8 else 0) + (4 if flg & 1 else 0)
        while p + 4 <= len(pay):
            w = struct.unpack_from("<I", pay, p)[0]
            p += 4
            if w == 0:
                break
            n = w & 0x7FFFFFFF
            if w & 0x80000000:
                raw += n
            else:
                comp += n
                nblk += 1
                if nblk <= seq_sample:
                    sampled_bytes += n
                    sampled_seq += _lz4_seq_count(pay[p:p + n])
            p += n + (4 if flg & 0x10 else 0)
    seq = int(round(comp * sampled_seq / sampled_bytes)) if sampled_bytes else 0
    return {"raw_block_bytes": raw, "comp_block_bytes": comp, "comp_blocks": nblk, "sequences_est": seq,
            "comp_block_decoded": max(0, lz4_out - raw)}


def host_threads() -> int:
    """Host cores this process may use: the pool's CPU share where the box
    sets one (OMP_NUM_THREADS = 16 per GPU there), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    aff = len(os.sched_getaffinity(0))
    return max(1, min(int(env), aff) if env and env.isdigit() else aff)


def gen_partitions(partitions, seg_bytes, kw, torch, device, threads=None):
    """Generate each partition's segment on the host (parallel, the GIL is
    released inside librpgen) and copy it into one device buffer.  Returns
    (data, offsets, batch counts, partition 0's host copy)."""
    n = len(partitions)
    data = torch.empty(n * seg_bytes + 256, dtype=torch.uint8, device=device)
    counts = [0] * n
    host_first = [None]
    lock = threading.Lock()
    sem = threading.Semaphore(threads or host_threads())
    errors = []

    def work(i, p):
        try:
            with sem:
                buf = np.empty(seg_bytes, dtype=np.uint8)
                counts[i] = synth.gen_segment(buf, p, **kw)
                with lock:
                    data[i * seg_bytes:(i + 1) * seg_bytes].copy_(torch.from_numpy(buf), non_blocking=False)
                    if i == 0:
                        host_first[0] = buf
        except Exception as e:  # surfaced after the join
            errors.append(e)
    ths = [threading.Thread(target=work, args=(i, p)) for i, p in enumerate(partitions)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if errors:
        raise errors[0]
    offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(seg_bytes)
    return data, offs, counts, host_first[0]


def cpu_baseline_c1(host_seg, seconds_budget=15.0):
    """The oracle's CPU restatement (SSE4.2 crc32c + record walk), timed on
    this box's host cores over a bounded sample of the same workload."""
    from oracle import oracle as O
    cores = host_threads()
    sample = host_seg[:CPU_C1_SAMPLE]
    # split the sample into `cores` slices on batch boundaries (16 KiB grid)
    per = max((sample.size // BATCH_BYTES) // cores, 1) * BATCH_BYTES
    cores = max(1, min(cores, sample.size // per))
    offs = np.arange(cores + 1, dtype=np.uint64) * np.uint64(per)
    sample = np.ascontiguousarray(sample[: int(offs[-1])])
    one = np.ascontiguousarray(sample[:per])
    nb1, s1, b1 = O.baseline_validate(one, [0, per], 1)
    reps, total_b, total_s = 0, 0, 0.0
    while total_s < seconds_budget and reps < 20:
        nb, s, b = O.baseline_validate(sample, offs, cores)
        total_b += b
        total_s += s
        reps += 1
    one_core = b1 / max(s1, 1e-9) / 1e9
    return {
        "value": round(total_b / max(total_s, 1e-9) / 1e9, 3),
        "unit": "GB/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{sample.size >> 20} MiB of the C1 workload (partition 0), header_crc + batch CRC32C (SSE4.2) "
                  f"+ record walk, {cores} pinned-per-core threads x {reps} reps",
        "one_core_GBs": round(one_core, 3),
        "host_logical_cpus": os.cpu_count(),
        "all_host_cpus_linear_estimate_GBs": round(one_core * (os.cpu_count() or 1), 1),
    }


def cpu_baseline_decode(host_seg, positions, seconds_budget=12.0, gz_zstd=False):
    """liblz4 1.9.3 / libsnappy 1.1.8 (the reference's codec libraries; for
    C6 also zlib 1.2.11 and libzstd 1.4) over the complete batches of one
    segment: stored crc + uncompress (the reference's driver loops) + decoded
    crc, one thread per core."""
    from oracle import oracle as O
    cores = host_threads()
    pos = np.asarray(positions, dtype=np.uint64)
    reps, tb, td, ts = 0, 0, 0, 0.0
    while ts < seconds_budget and reps < 200:
        s, b, d = O.baseline_decode(host_seg, pos, cores)
        tb, td, ts, reps = tb + b, td + d, ts + s, reps + 1
    sub = pos[: max(1, len(pos) // 8)]
    r1, b1, d1, s1 = 0, 0, 0, 0.0
    while s1 < 3.0 and r1 < 50:
        s, b, d = O.baseline_decode(host_seg, sub, 1)
        b1, d1, s1, r1 = b1 + b, d1 + d, s1 + s, r1 + 1
    return {
        "value": round(tb / max(ts, 1e-9) / 1e9, 3),
        "unit": "GB/s (stored bytes)",
        "decoded_GBs": round(td / max(ts, 1e-9) / 1e9, 3),
        "cores": cores,
        "kind": "reference",
        "sample": f"{len(pos)} batches ({tb // max(reps, 1) >> 20} MiB stored) of partition 0"
                  + (f"-{C6_CPU_PARTS - 1}" if gz_zstd else "") + ": stored crc + "
                  f"liblz4 LZ4F_decompress / libsnappy RawUncompress (lz4_frame_compressor.cc:123-200 / "
                  f"snappy_java_compressor.cc:76-129 loops)"
                  + (" / zlib inflate twice (gzip_compressor.cc:161-230) / libzstd ZSTD_decompressStream "
                     "(stream_zstd.cc:152-178)" if gz_zstd else "")
                  + f" + decoded crc, {cores} threads x {reps} reps; record walk not included",
        "one_core_GBs": round(b1 / max(s1, 1e-9) / 1e9, 3),
        "one_core_decoded_GBs": round(d1 / max(s1, 1e-9) / 1e9, 3),
        "host_logical_cpus": os.cpu_count(),
    }


def sized_outputs(eng, plat, data, offs, flags, nseg, est_batches):
    """Outputs sized from the job's own totals (a probe run)."""
    nb, nrec, ndec = est_batches, est_batches * 8, int(offs[-1]) * 2
    for _ in range(4):
        out = eng.alloc_outputs(nseg, nb + 16, nrec + 16, ndec + 4096)
        eng.submit(data, offs, out, flags)
        plat.sync()
        t = out.totals_host()
        if int(t["overflow"]) == 0:
            return out
        nb = max(nb, int(t["batch_capacity_needed"]))
        nrec = max(nrec, int(t["record_capacity_needed"]))
        ndec = max(ndec, int(t["decoded_capacity_needed"]))
        del out
    raise RuntimeError("output sizing did not converge")


def run_compressed(name, kw, n_parts, seg_bytes, args, plat, eng, abi, desc, extra_flags=0):
    """One compressed workload stanza (C2 / C5 / C6) on this GPU."""
    torch, device = plat.torch, plat.device
    t0 = time.time()
    data, offs, counts, host_first = gen_partitions(list(range(n_parts)), seg_bytes, kw, torch, device)
    log(f"[{name}] generated {n_parts} x {seg_bytes >> 20} MiB ({sum(counts)} batches) in {time.time() - t0:.1f}s")
    flags = abi.JOB_CRC | abi.JOB_PARSE | abi.JOB_DECODE | extra_flags
    d_offs = torch.from_numpy(offs.view(np.int64)).to(device)
    out = sized_outputs(eng, plat, data, offs, flags, n_parts, int(offs[-1]) // 4096 + 4096)
    # C6's step is ~0.3 s (serial gzip / zstd members): fewer timed steps
    steps = max(1, min(args.steps, 5) if name == "c6" else args.steps)
    for _ in range(min(args.warmup, 1) if name == "c6" else args.warmup):
        eng.submit(data, offs, out, flags, d_seg_offsets=d_offs)
    plat.sync()
    h = out.to_host()
    b = h.batches
    f = b["flags"]
    comp = (f & abi.F_COMPRESSED) != 0
    dec_ok = comp & ((f & abi.F_CODEC_OK) != 0)
    stored = int(np.sum(b["size_bytes"].astype(np.int64)))
    comp_in = int(np.sum(b["size_bytes"].astype(np.int64)[dec_ok] - abi.HEADER_SIZE))
    decoded = int(np.sum(b["decoded_len"].astype(np.int64)[dec_ok]))
    n_rec = int(h.totals["n_records"])
    # size-independent parity properties of the measured job
    crc_ok = (f & abi.F_CRC_OK) != 0
    parity = {
        "batches": int(len(b)),
        "compressed": int(np.sum(comp)),
        "codec_ok": int(np.sum(dec_ok)),
        "crc_ok": int(np.sum(crc_ok)),
        "parse_ok": int(np.sum((f & abi.F_PARSE_OK) != 0)),
        "overflow": int(h.totals["overflow"]),
        "discovery_rewalks": int(h.totals["n_rewalks"]),
        "records_eq_sum_parsed": bool(n_rec >= int(np.sum(b["records_parsed"].astype(np.int64)))),
        "terminal_errc": {int(k): int(v) for k, v in zip(*np.unique(h.summaries["terminal_errc"], return_counts=True))},
    }
    if name == "c2":
        parity["all_valid"] = bool(np.all(crc_ok) and np.all(dec_ok) and np.all(f & abi.F_PARSE_OK))
    positions = b["file_pos"][(b["segment"] == 0) & ((f & abi.F_COMPLETE) != 0)]
    cpu_host = host_first
    if name == "c6" and n_parts >= C6_CPU_PARTS:
        cpu_host = data[: int(offs[C6_CPU_PARTS])].cpu().numpy()
        sel = (b["segment"] < C6_CPU_PARTS) & ((f & abi.F_COMPLETE) != 0)
        positions = b["file_pos"][sel] + offs[b["segment"][sel].astype(np.int64)]
    per_codec = None
    if name == "c6":
        codec = b["attrs"] & 7
        per_codec = {str(c): {"batches": int(np.sum(codec == c)), "codec_ok": int(np.sum(dec_ok & (codec == c))),
                              "decoded_bytes": int(np.sum(b["decoded_len"].astype(np.int64)[dec_ok & (codec == c)]))}
                     for c in (1, 2, 3, 4)}
    n_batches = int(len(b))
    stored_payload = int(np.sum(b["size_bytes"].astype(np.int64) - abi.HEADER_SIZE))
    lz4c = None
    if args.stats_out and host_first is not None:
        # partition 0's LZ4 block composition, scaled to the job by stored bytes
        s0 = (b["segment"] == 0) & dec_ok
        lz4c = lz4_composition(host_first, b["file_pos"][s0], b["size_bytes"][s0], b["attrs"][s0],
                               b["decoded_len"][s0].astype(np.int64))
        scale = stored / max(1, int(np.sum(b["size_bytes"].astype(np.int64)[b["segment"] == 0])))
        lz4c = {k: int(round(v * scale)) for k, v in lz4c.items()}
        lz4c["sample"] = "partition 0, scaled by stored bytes"
    del h, b, f
    eng.set_timing(True)
    plat.sync()
    t1 = time.perf_counter()
    for _ in range(steps):
        eng.submit(data, offs, out, flags, d_seg_offsets=d_offs)
    plat.sync()
    el = (time.perf_counter() - t1) / steps
    tm = eng.last_timings()
    eng.set_timing(False)
    dec_ms = tm["decode"]
    # decode stage (k_decode .. k_content_apply): compressed payload read
    # once + decoded bytes written once
    dec_alg = comp_in + decoded
    # whole pipeline, SURVEY §8(d) C2/C5 bytes per unit: every stored byte
    # read once (compressed payloads, uncompressed payloads, headers) +
    # decoded bytes written once + the index (48 B per record, 64 B per
    # batch result); the CRC / walk of the decoded bytes is not counted again
    whole_alg = stored + decoded + IDX_BYTES_PER_RECORD * n_rec + RESULT_BYTES_PER_BATCH * n_batches
    traffic, kernels_traffic = profiled_traffic("decode_traffic.json", name,
                                                DECODE_KERNELS + (MEMBER_KERNELS if name == "c6" else ()))
    cpu = None
    if not args.no_cpu_baseline and len(positions):
        try:
            cpu = cpu_baseline_decode(cpu_host, positions, gz_zstd=(name == "c6"))
        except Exception as e:  # a baseline failure must not cost the GPU measurement
            cpu = failure(f"{name} cpu baseline", e)
    write_stats(args, name, {"stored": stored, "stored_payload": stored_payload, "compressed_in": comp_in,
                             "decoded": decoded, "batches": n_batches,
                             "compressed_batches": parity["compressed"], "records": n_rec, "lz4": lz4c})
    st = {
        "workload_id": name.upper(),
        "workload": desc,
        "partitions": n_parts,
        "segment_bytes": seg_bytes,
        "stored_bytes": stored,
        "generated_bytes": int(offs[-1]),
        "generated_batches": int(sum(counts)),
        "reachable_note": "stored_bytes / batches count the batches the parser chain reaches; a chain ends at an "
                          "injected header fault (storage/parser.cc semantics), so generated bytes past it are "
                          "not batches" if int(sum(counts)) != n_batches else "every generated batch is reached",
        "decoded_bytes": decoded,
        "batches": n_batches,
        "records": n_rec,
        "ms_per_step": round(el * 1e3, 3),
        "steps": steps,
        "stored_GBps": round(stored / el / 1e9, 2),
        "decoded_GBps": round(decoded / el / 1e9, 2),
        "batches_per_s": round(n_batches / el, 1),
        "hbm_fraction_whole_pipeline": round(whole_alg / el / 1e9 / HBM_PEAK_GBS, 4),
        "whole_alg_bytes": whole_alg,
        "whole_alg_def": "stored + decoded + 48 B/record + 64 B/batch (SURVEY §8(d))",
        "stage_ms": {k: round(v, 4) for k, v in tm.items()},
        "roofline": {
            "bound": "hbm",
            "kernel": "decode stage (k_decode .. k_content_apply)",
            "achieved": round(dec_alg / (dec_ms * 1e-3) / 1e9, 1) if dec_ms > 0 else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(dec_alg / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if dec_ms > 0 else None,
            "traffic": traffic,
            "alg_bytes_per_launch": dec_alg,
            "alg_def": "compressed payload read + decoded bytes written",
            "kernel_ms": round(dec_ms, 4),
            "traffic_source": kernels_traffic.get("source") if kernels_traffic else None,
            "kernels_traffic": kernels_traffic,
        },
        "parity": parity,
        "cpu_baseline": cpu,
    }
    if per_codec is not None:
        st["per_codec"] = per_codec
        # gzip / zstd members decode in the member pass, which runs inside the
        # resolve_plan stage (it sizes their arena slots, as the reference's
        # buffer_for_input does)
        gz_zs = sum(per_codec[c]["decoded_bytes"] for c in ("1", "4"))
        rp = tm["resolve_plan"]
        # zstd members parsed in the member pass execute in k_zexec, inside
        # the decode stage: the rate is taken over both stages (a lower
        # bound: the decode stage also runs the lz4 / snappy pieces)
        both = rp + dec_ms
        st["member_pass"] = {"stage": "resolve_plan (gzip: members >= 16 KiB in chunks from speculative block "
                                      "starts, k_gzsplan / k_gzsfind / k_gzsdecode / k_gzsresolve, the rest serial "
                                      "in k_members_first; zstd beside them on a side stream: k_zplan, k_zlits, "
                                      "k_zparse, k_zfallback) + decode (k_zexec executes the parsed zstd members)",
                             "ms": round(rp, 3), "decoded_bytes": gz_zs,
                             "gzip_decoded_bytes": per_codec["1"]["decoded_bytes"],
                             "zstd_decoded_bytes": per_codec["4"]["decoded_bytes"],
                             "decoded_GBps": round(gz_zs / (both * 1e-3) / 1e9, 3) if both > 0 else None,
                             "decoded_GBps_def": "gzip + zstd decoded bytes / (resolve_plan + decode stage ms)"}
    del out, data, d_offs, cpu_host
    plat.empty_cache()
    return st


def job_digest(abi, res) -> str:
    """sha256 over every compared field of a job's batch results and record
    index (the fields the GPU parity tests compare with the oracle)."""
    import hashlib
    h = hashlib.sha256()
    for f in abi.BATCH_COMPARE_FIELDS:
        h.update(np.ascontiguousarray(res.batches[f]).tobytes())
    for f in abi.RECORD_COMPARE_FIELDS:
        h.update(np.ascontiguousarray(res.records[f]).tobytes())
    return h.hexdigest()


def run_h2d(args, plat, eng, abi, data, seg_bytes, n_parts, flags, ref):
    """H2D-inclusive rate (rpgpu_validate_host): the same C1 partitions,
    host-resident in pinned memory, copied to the device in double-buffered
    staging groups on a copy stream while the previous group validates, with
    the batch results, record index and summaries returned to host arrays
    (storage/log_replayer.cc:95-114 reads segments from the file into
    memory).  Not `value` (device-resident); reported beside
    it.  `ref` = the device job's (n_batches, n_records, job_digest)."""
    host = plat.host_segments(data, seg_bytes, n_parts)
    total = seg_bytes * n_parts
    r = eng.validate_host(host, flags)  # warm-up: staging slots allocated
    b = r.batches
    counts_ok = bool(len(b) == ref[0] and len(r.records) == ref[1] and np.all(b["flags"] & abi.F_CRC_OK)
                     and np.all(b["flags"] & abi.F_PARSE_OK) and int(r.totals["overflow"]) == 0)
    same = bool(ref[2] is not None and job_digest(abi, r) == ref[2])
    del r, b
    reps = max(1, min(args.steps, 3))
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = eng.validate_host(host, flags)
        times.append(time.perf_counter() - t0)
        del r
    del host
    best, mean = min(times), sum(times) / len(times)
    return {
        "path": "rpgpu_validate_host (pinned host segments -> H2D on a copy stream, double-buffered groups, "
                "results + record index back to host arrays)",
        "group_bytes": max(HOST_GROUP_BYTES, seg_bytes),
        "bytes": total,
        "reps": reps,
        "GBps": round(total / mean / 1e9, 2),
        "GBps_best": round(total / best / 1e9, 2),
        "ms_per_job": round(mean * 1e3, 2),
        # counts and verdict bits, and every compared field of the batch
        # results and the record index (sha256) against the device job's
        "parity": {"counts_and_flags_match": counts_ok, "batch_results_and_record_index_identical": same},
    }


def run_stanza(name, *a, **kw):
    """A compressed-workload stanza: a failure there is reported in its
    stanza instead of costing the headline line."""
    try:
        return run_compressed(name, *a, **kw)
    except Exception as e:
        return failure(name, e)


def _pick(d, keys):
    return {k: d[k] for k in keys if d is not None and k in d}


def compact_stanza(st):
    """The fields of a stanza that ride on the JSON line.  The driver keeps
    only the last 8 KB of stdout, so the per-kernel traffic tables, codec
    splits and long descriptions go to --detail-out instead (the line names
    the committed profile they come from)."""
    if st is None or "error" in st:
        return st
    rf = st.get("roofline") or {}
    out = _pick(st, ("workload_id", "ms_per_step", "stored_GBps", "decoded_GBps", "batches_per_s",
                     "hbm_fraction_whole_pipeline", "stage_ms"))
    out["roofline"] = _pick(rf, ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic", "kernel_ms",
                                 "alg_bytes_per_launch", "traffic_source"))
    p = st.get("parity") or {}
    out["parity"] = _pick(p, ("batches", "codec_ok", "crc_ok", "parse_ok", "overflow", "all_valid",
                              "records_eq_sum_parsed"))
    out["cpu_baseline"] = _pick(st.get("cpu_baseline"), ("value", "unit", "decoded_GBs", "cores", "kind", "error"))
    if "member_pass" in st:
        out["member_pass"] = _pick(st["member_pass"], ("ms", "decoded_bytes", "decoded_GBps"))
    return out


STANZAS = {
    "c2": (lambda: synth.C2, lambda: (C2_PARTS, C2_SEG),
           "C2: 8 partitions x 1.5 GiB disk segments of LZ4 frames (64 KiB blocks, content size; 10% linked, "
           "10% content checksum), decoded batches uniform 64 KiB..1 MiB, payload thirds random / alnum / "
           "JSON-like (seed 0xC2): discover + header_crc + crc + LZ4F decode + decoded crc/header_crc + record walk"),
    "c6": (lambda: synth.C6, lambda: (C5_PARTS, C5_SEG),
           "C6 (C5 + gzip / zstd): 128 partitions x 64 MiB, log-uniform 200 B..1 MiB batches, none 32 / gzip 10 / "
           "lz4 24 / snappy-java 12 / raw snappy 12 / zstd 10, every codec decoded on the device, 1% payload + "
           "0.2% header bit flips, 0.1% zeroed headers, truncated tails (seed 0xC6)"),
    "c5": (lambda: synth.C5, lambda: (C5_PARTS, C5_SEG),
           "C5: 128 partitions x 64 MiB, log-uniform 200 B..1 MiB batches, none 40 / lz4 30 / snappy-java 15 / "
           "raw snappy 15, 1% payload + 0.2% header bit flips, 0.1% zeroed headers, truncated tails (seed 0xC5)"),
}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seg-gib", type=float, default=SEG_BYTES / (1 << 30))
    ap.add_argument("--partitions", type=int, default=PARTITIONS_PER_GPU)
    ap.add_argument("--chunk-kib", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", choices=["bitmap", "index", "records"], default="bitmap",
                    help="what travels to rank 0 each step at N > 1: bitmaps + summaries (default), + batch results, "
                         "+ batch results and the per-record index")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl (RCCL over xGMI, the product path); gloo stages the gather through host memory "
                         "(a rehearsal of the N > 1 path, e.g. several ranks on one card)")
    ap.add_argument("--check-gather", action="store_true",
                    help="at N > 1, after the timed region: rank 0 runs ONE job over every partition and compares the "
                         "gathered verdicts, bitmaps, batch results, record index and segment indexes with it")
    ap.add_argument("--no-parse", action="store_true", help="CRC only (diagnostic; not the headline workload)")
    ap.add_argument("--no-index", action="store_true", help="skip the segment-index rebuild measurement")
    ap.add_argument("--batch-bytes", type=int, default=BATCH_BYTES,
                    help="size_bytes per batch (diagnostic; the headline workload is 16 KiB)")
    ap.add_argument("--stats-out", default="",
                    help="write each workload's byte counts (JSON) here, for scripts/parse_traffic.py")
    ap.add_argument("--workloads", default="c1,h2d,c2,c5,c6",
                    help="c1 is the headline; h2d (the host path over c1's partitions) and the c2/c5/c6 stanzas run "
                         "at N = 1 only; a run without c1 is a diagnostic (per-workload profiles)")
    ap.add_argument("--no-h2d", action="store_true", help="skip the H2D-inclusive host-path stanza")
    ap.add_argument("--detail-out", default="",
                    help="write the full stanzas (per-kernel traffic tables, codec splits, descriptions) here; the "
                         "JSON line carries the compact form")
    return ap.parse_args(argv)


def main(argv=None, platform=None):
    args = parse_args(argv)
    workloads = [w for w in args.workloads.split(",") if w]

    import torch.distributed as dist
    from redpanda_amd import abi

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    plat = (platform or CudaPlatform)(local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=plat.device)
        else:
            dist.init_process_group("gloo")
    try:
        eng = plat.engine()
        c1 = run_c1(args, plat, dist, eng, abi, world, rank) if "c1" in workloads else None
        if c1 is None and world > 1:
            raise SystemExit("--gpus N > 1 runs the headline workload (c1)")

        extra = {}
        if world == 1:
            for name in ("c2", "c6", "c5"):
                if name in workloads:
                    kw, size, desc = STANZAS[name]
                    parts, seg = size()
                    extra[name] = run_stanza(name, kw(), parts, seg, args, plat, eng, abi, desc)

        if rank == 0:
            if args.detail_out:
                try:
                    with open(args.detail_out, "w") as f:
                        json.dump({"c1": c1, **extra}, f, indent=1, default=str)
                except Exception as e:
                    failure("detail-out", e)
            roof = dict(c1["roofline"]) if c1 else None
            if roof:
                roof.pop("kernels_traffic", None)  # per-kernel tables: --detail-out / the committed profile
            line = {
                "metric": "validated+decoded batch GB/s per GPU and whole node; % of HBM peak",
                "value": c1["value"] if c1 else None,
                "unit": "GB/s",
                "n_gpus": world,
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": c1["ms_per_step"] if c1 else None,
                "higher_is_better": True,
                "scaling": "weak",
                "vs_baseline": None,
                "dtype": "u8",
                "data": "synthetic (seeded mt19937_64, reference random_batch recipe), device-resident",
                "config": {**(c1["config"] if c1 else {"workload": "diagnostic run without the headline (c1) workload"}),
                           **({"h2d": c1["h2d"]} if c1 and c1.get("h2d") is not None else {}),
                           **{k: compact_stanza(v) for k, v in extra.items()}},
                "roofline": roof,
                "cpu_baseline": _pick(c1["cpu_baseline"], ("value", "unit", "cores", "kind", "sample", "one_core_GBs",
                                                           "host_logical_cpus", "error")) if c1 else None,
            }
            print(json.dumps(line, separators=(",", ":")), flush=True)
    finally:
        if world > 1:
            dist.destroy_process_group()


def check_gather(args, plat, dist, eng, abi, out, index_res, parts, nb, n_records, world, rank, flags, seg_bytes):
    """--check-gather: the gathered job at rank 0 against ONE single-process
    job over every partition (global partition order) on rank 0's device.
    Every rank takes part in the gathers; rank 0 returns the comparison."""
    from redpanda_amd.shard import gather_job_verdicts, gather_records, gather_segment_index
    v = gather_job_verdicts(out.summaries, out.bitmap, nb, parts, rank, world, dist)
    g = gather_records(out.batches[: nb * abi.BATCH_RESULT.itemsize],
                       out.records[: n_records * abi.RECORD_INDEX.itemsize], out.summaries, parts, rank, world, dist)
    gi = gather_segment_index(*index_res, parts, rank, world, dist) if index_res is not None else None
    if rank != 0:
        return None
    all_parts = list(range(args.partitions * world))
    data, offs, counts, _ = gen_partitions(all_parts, seg_bytes, dict(synth.C1, batch_bytes=args.batch_bytes),
                                           plat.torch, plat.device)
    n_all = int(sum(counts))
    ref = eng.alloc_outputs(len(all_parts), n_all + 16, n_all * 32 + 16, 1)
    eng.submit(data, offs, ref, flags)
    plat.sync()
    r = ref.to_host()
    res = {"partitions": len(all_parts)}
    res["summaries"] = bool(all(np.array_equal(v["summaries"][fld], r.summaries[fld]) for fld in SUMMARY_JOB_FIELDS))
    bits = np.unpackbits(r.bitmap.view(np.uint8), bitorder="little") if r.bitmap is not None else None
    ok_bits = bits is not None
    for key, got in v["bitmaps"].items():
        if not ok_bits:
            break
        want = np.concatenate([bits[int(r.summaries["first_batch"][p]):
                                    int(r.summaries["first_batch"][p]) + int(r.summaries["n_batches"][p])]
                               for p in key])
        ok_bits = np.array_equal(got, want)
    res["bitmaps"] = bool(ok_bits)
    gb, gr = g["batches"], g["records"]
    res["batches"] = bool(len(gb) == len(r.batches) and all(
        np.array_equal(gb[fld], r.batches[fld]) for fld in abi.BATCH_COMPARE_FIELDS if fld != "decoded_off"))
    res["records"] = bool(len(gr) == len(r.records) and all(
        np.array_equal(gr[fld], r.records[fld]) for fld in abi.RECORD_COMPARE_FIELDS))
    res["n_batches"], res["n_records"] = int(len(gb)), int(len(gr))
    if gi is not None:
        ri = eng.index_to_host(*eng.segment_index(ref, [0] * len(all_parts)), n_segments=len(all_parts))
        res["index"] = bool(sorted(gi) == all_parts and all(
            all(int(gi[p][0][fld]) == int(ri[p][0][fld]) for fld in abi.INDEX_STATE.names if fld != "first_entry")
            and all(np.array_equal(gi[p][k], ri[p][k]) for k in (1, 2, 3)) for p in all_parts))
    res["consistent"] = bool(all(res[k] for k in ("summaries", "bitmaps", "batches", "records"))
                             and res.get("index", True))
    del ref, data, r
    plat.empty_cache()
    return res


def run_c1(args, plat, dist, eng, abi, world, rank):
    """The headline workload (C1 per GPU; C3 across ranks): returns the
    fields of the JSON line it owns."""
    from redpanda_amd.shard import as_bytes, gather_bytes, gather_job_verdicts, gather_records, gather_sizes, \
        partitions_for_rank
    torch, device = plat.torch, plat.device
    comm = plat.comm_device(args.dist_backend)
    seg_bytes = int(args.seg_gib * (1 << 30)) // BATCH_BYTES * BATCH_BYTES
    parts = partitions_for_rank(args.partitions * world, world, rank)
    t0 = time.time()
    data, offs, counts, host_first = gen_partitions(parts, seg_bytes, dict(synth.C1, batch_bytes=args.batch_bytes),
                                                    torch, device)
    n_batches = int(sum(counts))
    log(f"[rank {rank}] generated {len(parts)} x {seg_bytes >> 20} MiB, {n_batches} batches in {time.time() - t0:.1f}s")

    flags = abi.JOB_CRC | (0 if args.no_parse else abi.JOB_PARSE)
    rec_per_batch = 32
    out = eng.alloc_outputs(len(parts), n_batches + 16, n_batches * rec_per_batch, 1)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(device)
    chunk = args.chunk_kib << 10
    # the gather payload: validity bitmaps + segment summaries, plus the
    # per-batch results (--gather index) or the results and the per-record
    # index (--gather records)
    payload = [out.bitmap, out.summaries]
    if args.gather in ("index", "records"):
        payload.append(out.batches[: n_batches * abi.BATCH_RESULT.itemsize])
    if args.gather == "records":
        eng.submit(data, offs, out, flags, chunk, d_seg_offsets=d_offs)
        plat.sync()
        n_records_est = int(out.totals_host()["n_records"])
        payload.append(out.records[: n_records_est * abi.RECORD_INDEX.itemsize])
    # the gather's per-rank lengths are fixed for the run: negotiated once,
    # outside the timed loop (no host sync per step with nccl)
    sizes = [gather_sizes(as_bytes(t), world, dist) for t in payload] if world > 1 else None

    def step():
        eng.submit(data, offs, out, flags, chunk, d_seg_offsets=d_offs)
        if world > 1:
            # the one exchange: to rank 0
            for t, sz in zip(payload, sizes):
                gather_bytes(as_bytes(t), rank, world, dist, sizes=sz)

    for _ in range(args.warmup):
        step()
    plat.sync()
    # correctness of the measured workload (size-independent properties)
    h = out.to_host()
    nb = len(h.batches)
    all_ok = bool(nb == n_batches and (args.no_parse or np.all(h.batches["flags"] & abi.F_PARSE_OK))
                  and np.all(h.batches["flags"] & abi.F_CRC_OK) and h.totals["overflow"] == 0)
    bm_ok = bool(np.all(h.bitmap[: nb // 64] == np.uint64(0xFFFFFFFFFFFFFFFF)))
    n_records = int(h.totals["n_records"])
    gathered = None
    if world > 1:
        # the gathered job picture on rank 0: every partition checkpointed at its end
        g = gather_job_verdicts(out.summaries, out.bitmap, nb, parts, rank, world, dist)
        if rank == 0:
            all_ok = bool(all_ok and np.all(g["summaries"]["has_checkpoint"] == 1)
                          and np.all(g["summaries"]["first_bad"] == g["summaries"]["n_batches"]))
        if args.gather == "records":
            gr = gather_records(out.batches[: nb * abi.BATCH_RESULT.itemsize],
                                out.records[: n_records * abi.RECORD_INDEX.itemsize], out.summaries, parts, rank,
                                world, dist)
            if rank == 0:
                b, r = gr["batches"], gr["records"]
                ok = bool(len(r) == int(np.sum(b["records_parsed"].astype(np.int64)))
                          and np.all(np.diff(b["index_base"].astype(np.int64)) >= 0)
                          and np.all(np.diff(r["batch"].astype(np.int64)) >= 0))
                gathered = {"batches": int(len(b)), "records": int(len(r)), "consistent": ok}
        if rank == 0:
            gathered = dict(gathered or {}, bytes_per_step=int(sum(max(sz) * world for sz in sizes)),
                            backend=args.dist_backend)
    payload_bytes = int(np.sum(h.batches["size_bytes"].astype(np.int64) - abi.HEADER_SIZE))
    seg_total = int(np.sum(h.batches["size_bytes"].astype(np.int64)))
    del h
    if rank == 0:
        write_stats(args, "c1", {"stored": seg_total, "stored_payload": payload_bytes, "compressed_in": 0, "decoded": 0,
                                 "batches": n_batches, "compressed_batches": 0, "records": n_records})

    eng.set_timing(True)
    if world > 1:
        dist.barrier()
    plat.sync()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        step()
    plat.sync()
    if world > 1:
        dist.barrier()
    t2 = time.perf_counter()
    eng.set_timing(False)
    tm = eng.last_timings()
    elapsed = t2 - t1
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=comm)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        tb = torch.tensor([seg_total, n_batches], dtype=torch.float64, device=comm)
        dist.all_reduce(tb, op=dist.ReduceOp.SUM)
        job_bytes, job_batches = float(tb[0].item()), float(tb[1].item())
    else:
        job_bytes, job_batches = float(seg_total), float(n_batches)
    ms_per_step = elapsed / args.steps * 1e3
    value = job_bytes * args.steps / elapsed / 1e9

    # Everything below is after the headline's timed region: each leg
    # reports a failure in its own field instead of costing the line.

    # roofline of the dominant kernel (k_validate: CRC32C of every stored
    # payload): algorithmic bytes per launch = payload read once + 128 B per
    # batch result (descriptor read + verdict written, counted once).  The
    # record walk runs in k_walk (index writes + the result struct), reported
    # beside it.
    alg = payload_bytes + 128 * n_batches
    v_ms = tm["validate"]
    achieved = alg / (v_ms * 1e-3) / 1e9 if v_ms > 0 else None
    walk_alg = abi.RECORD_INDEX.itemsize * n_records + 128 * n_batches
    w_ms = tm.get("walk", 0.0)
    # SURVEY §8(d) C1 bytes per unit: segment bytes read once + 48 B per
    # record + 64 B per batch
    whole_alg = seg_total + IDX_BYTES_PER_RECORD * n_records + RESULT_BYTES_PER_BATCH * n_batches
    _, c1_traffic = profiled_traffic("validate_traffic.json", "c1", ("k_validate", "k_walk"))
    traffic = c1_traffic.get("k_validate", {}).get("bytes") if c1_traffic else None

    # segment sparse-index rebuild (segment_index::maybe_track over the
    # recovered batches, §8(f) row 2): timed separately on its own stream,
    # after the headline region; not part of `value`
    index, index_res = None, None
    if not args.no_index:
        try:
            bases = [0] * len(parts)
            ms, index_res = plat.time_on_side_stream(
                lambda st: eng.segment_index(out, bases, stream=st),
                lambda st, prev: eng.segment_index(out, bases, stream=st, outputs=prev), 5)
            ix = eng.index_to_host(*index_res, n_segments=len(parts))
            n_entries = int(sum(int(r[0]["n_entries"]) for r in ix))
            gidx = None
            if world > 1:
                # the job's indexes at rank 0 (gather of the used entries only)
                from redpanda_amd.shard import gather_segment_index
                gi = gather_segment_index(*index_res, parts, rank, world, dist)
                if rank == 0:
                    gidx = {"partitions": len(gi), "entries": int(sum(int(v[0]["n_entries"]) for v in gi.values()))}
            index = {"kernel": "k_idx_cut+k_idx_cand+k_idx_resolve+k_idx_emit", "ms": round(ms, 4),
                     "step": abi.INDEX_DEFAULT_STEP, "entries": n_entries,
                     "tracked": int(sum(int(r[0]["tracked"]) for r in ix)), "gathered_at_rank0": gidx,
                     "note": "piece-parallel (1024-batch pieces, candidate first entries, serial resolve); "
                             "outputs preallocated, timed region = the four kernels + workspace memset"}
            del ix
        except Exception as e:
            index = failure("segment index", e)
            if world > 1:
                raise  # a rank that left the gather would hang the others

    gcheck = None
    if world > 1 and args.check_gather:
        gcheck = check_gather(args, plat, dist, eng, abi, out, index_res, parts, nb, n_records, world, rank, flags,
                              seg_bytes)

    cpu = None
    if rank == 0 and not args.no_cpu_baseline and host_first is not None:
        try:
            cpu = cpu_baseline_c1(host_first)
        except Exception as e:
            cpu = failure("c1 cpu baseline", e)
    dev_digest = None
    if world == 1 and not args.no_h2d and "h2d" in args.workloads.split(","):
        try:
            dev_digest = job_digest(abi, out.to_host())
        except Exception:
            dev_digest = None
    # release the C1 job's outputs before the host path allocates its own
    del out, d_offs, payload, index_res
    plat.empty_cache()
    h2d = None
    if world == 1 and not args.no_h2d and "h2d" in args.workloads.split(","):
        try:
            h2d = run_h2d(args, plat, eng, abi, data, seg_bytes, len(parts), flags, (n_batches, n_records, dev_digest))
        except Exception as e:
            h2d = failure("h2d", e)
    del data
    plat.empty_cache()
    gather_desc = {"bitmap": "bitmaps+summaries", "index": "bitmaps+summaries+batch results",
                   "records": "bitmaps+summaries+batch results+record index"}[args.gather]
    coll = "RCCL" if args.dist_backend == "nccl" else "gloo (host-staged)"
    trace = committed_trace("k_validate")
    return {
        "value": round(value, 2),
        "ms_per_step": round(ms_per_step, 4),
        "h2d": h2d,
        "config": {
            "workload": "C1/C3: per GPU 8 partitions x 2 GiB disk segments of uncompressed 16 KiB batches "
                        "(seed 0xC1): discovery + header_crc + CRC32C + record walk/index + checkpoint",
            "segment_bytes": seg_bytes,
            "partitions_per_gpu": len(parts),
            "batches_per_gpu": n_batches,
            "records_per_gpu": n_records,
            "batch_bytes": args.batch_bytes,
            "batches_per_s": round(job_batches * args.steps / elapsed, 1),
            "parallelism": f"partition-sharded x{world}, {coll} gather of {gather_desc}",
            "gathered_records": gathered,
            "gather_check": gcheck,
            "parity": {"all_batches_valid": all_ok, "bitmap_all_ones": bm_ok},
            "stage_ms": {k: round(v, 4) for k, v in tm.items()},
            "hbm_fraction_whole_pipeline": round(value / world / HBM_PEAK_GBS, 4),
            "hbm_fraction_whole_pipeline_alg": round(whole_alg / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "whole_alg_def": "segment bytes + 48 B/record + 64 B/batch (SURVEY §8(d))",
            "segment_index": index,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_validate",
            "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            "traffic": traffic,
            "traffic_source": c1_traffic.get("source") if c1_traffic else None,
            "alg_bytes_per_launch": alg,
            "kernel_ms": round(v_ms, 4),
            "kernel_ms_def": "validate stage between HIP events on the launch stream, mean over the timed steps",
            # the COMMITTED rocprofv3 trace of the driver's command (taken on
            # the tree named by its tag, not in this run): its mean and the
            # fraction it implies, labelled as such
            "committed_trace": dict(trace, source="profiles/kernel_trace.json (committed; not this run)",
                                    frac_at_trace=round(alg / (trace["mean_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
            if trace else None,
            "walk": {"kernel": "k_walk", "kernel_ms": round(w_ms, 4), "alg_bytes_per_launch": walk_alg,
                     "achieved": round(walk_alg / (w_ms * 1e-3) / 1e9, 1) if w_ms > 0 else None},
            "kernels_traffic": c1_traffic,
        },
        "cpu_baseline": cpu,
    }


def committed_trace(kernel, fname="kernel_trace.json"):
    """The committed rocprofv3 --kernel-trace summary of the driver's bench
    command (scripts/trace_summary.py -> profiles/kernel_trace.json): the
    mean duration of `kernel`'s C1 launches and the tag it was taken on."""
    try:
        with open(os.path.join(ROOT, "profiles", fname)) as f:
            tj = json.load(f)
        k = tj["c1"][kernel]
        return {"tag": tj.get("tag"), "mean_ms": k["mean_ms"], "calls": k["calls"]}
    except Exception:
        return None


if __name__ == "__main__":
    main()
