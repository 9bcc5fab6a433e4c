#!/usr/bin/env python3
"""Diagnostic bench of the compressed configurations (BASELINE.json
configs[2] C2 and configs[4] C5); the headline bench.py stays on C1.

C2: LZ4 frames (blockIndependent, 64 KiB blocks, contentSize; liblz4 via the
generator), decoded batches log-uniform in 64 KiB..1 MiB, payload thirds of
random / alnum / repetitive JSON-like records.  C5: 200 B..1 MiB, codecs
none / lz4 / snappy, 1% payload corruption.  One step = the whole pipeline
with CRC | PARSE | DECODE over device-resident segments.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["c2", "c5"], default="c2")
    ap.add_argument("--partitions", type=int, default=8)
    ap.add_argument("--seg-mib", type=int, default=256)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()

    import torch
    from redpanda_amd import _lib, abi
    from redpanda_amd.engine import Engine

    dev = torch.device("cuda", 0)
    seg = args.seg_mib << 20
    if args.workload == "c2":
        kw = dict(seed=0xC2, batch_bytes=0, min_batch=64 << 10, max_batch=1 << 20, codec_mix=1 << abi.CODEC_LZ4)
    else:
        kw = dict(seed=0xC5, batch_bytes=0, min_batch=200, max_batch=1 << 20,
                  codec_mix=(1 << abi.CODEC_NONE) | (1 << abi.CODEC_LZ4) | (1 << abi.CODEC_SNAPPY),
                  corrupt_payload_ppm=10000)
    bufs = [None] * args.partitions
    t0 = time.time()

    def work(i):
        b = np.empty(seg, dtype=np.uint8)
        _lib.gen_segment(b, i, **kw)
        bufs[i] = b
    ths = [threading.Thread(target=work, args=(i,)) for i in range(args.partitions)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    host = np.concatenate(bufs)
    del bufs
    data = torch.from_numpy(host).to(dev)
    offs = np.arange(args.partitions + 1, dtype=np.uint64) * np.uint64(seg)
    print(f"generated {host.size >> 20} MiB in {time.time() - t0:.1f}s", file=sys.stderr)

    eng = Engine(0)
    flags = abi.JOB_CRC | abi.JOB_PARSE | abi.JOB_DECODE
    # size the outputs from a first run's totals
    probe = eng.alloc_outputs(args.partitions, host.size // abi.HEADER_SIZE + 16, 1, 1)
    eng.submit(data, offs, probe, flags)
    torch.cuda.synchronize()
    t = probe.to_host().totals
    nb, nrec, ndec = int(t["batch_capacity_needed"]), int(t["record_capacity_needed"]), int(t["decoded_capacity_needed"])
    del probe
    out = eng.alloc_outputs(args.partitions, nb + 16, nrec + 16, ndec + 64)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    for _ in range(args.warmup):
        eng.submit(data, offs, out, flags, d_seg_offsets=d_offs)
    torch.cuda.synchronize()
    h = out.to_host()
    f = h.batches["flags"]
    comp = (f & abi.F_COMPRESSED) != 0
    decoded_bytes = int(np.sum(h.batches["decoded_len"].astype(np.int64)[comp]))
    stored = int(np.sum(h.batches["size_bytes"].astype(np.int64)))
    ok = {
        "batches": int(len(f)),
        "codec_ok": int(np.sum((f & abi.F_CODEC_OK) != 0)),
        "compressed": int(np.sum(comp)),
        "crc_ok": int(np.sum((f & abi.F_CRC_OK) != 0)),
        "parse_ok": int(np.sum((f & abi.F_PARSE_OK) != 0)),
        "overflow": int(h.totals["overflow"]),
    }
    eng.set_timing(True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        eng.submit(data, offs, out, flags, d_seg_offsets=d_offs)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t1) / args.steps
    tm = eng.last_timings()
    eng.set_timing(False)
    dec_ms = tm["decode"]
    # k_decode algorithmic bytes: compressed payload read + decoded bytes written
    comp_in = int(np.sum(h.batches["size_bytes"].astype(np.int64)[comp] - abi.HEADER_SIZE))
    line = {
        "workload": args.workload,
        "stored_GBps": round(stored / el / 1e9, 2),
        "decoded_GBps": round(decoded_bytes / el / 1e9, 2),
        "ms_per_step": round(el * 1e3, 3),
        "stage_ms": {k: round(v, 4) for k, v in tm.items()},
        "k_decode_GBps_alg": round((comp_in + decoded_bytes) / (dec_ms * 1e-3) / 1e9, 1) if dec_ms else None,
        "stored_bytes": stored,
        "decoded_bytes": decoded_bytes,
        "ratio": round(decoded_bytes / max(comp_in, 1), 3),
        "verdicts": ok,
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
