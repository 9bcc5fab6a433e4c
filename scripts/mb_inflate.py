"""Microbenchmark of the device inflate (diagnostic): jobs of gzip-only
batches, timed per stage (plan = k_inflate_plan sizing pass, decode =
k_inflate)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import synth
from redpanda_amd import abi
from redpanda_amd.engine import Engine

eng = Engine(0)
F = abi.JOB_CRC | abi.JOB_PARSE | abi.JOB_DECODE
for codec, nseg, seg_mib, bmin, bmax in [(1, 1, 2, 1 << 20, 1 << 20), (1, 1, 2, 64 << 10, 64 << 10),
                                         (1, 16, 16, 1 << 20, 1 << 20), (1, 64, 16, 64 << 10, 256 << 10),
                                         (4, 1, 2, 1 << 20, 1 << 20), (4, 1, 2, 64 << 10, 64 << 10),
                                         (4, 16, 16, 1 << 20, 1 << 20), (4, 64, 16, 64 << 10, 256 << 10)]:
    w = [0] * 6
    w[codec] = 1
    segs = []
    for i in range(nseg):
        a = np.zeros(seg_mib << 20, np.uint8)
        synth.gen_segment(a, i, seed=77 + i, batch_bytes=0, min_batch=bmin, max_batch=bmax, weights=w,
                          size_uniform=True)
        segs.append(a)
    offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
    data = np.concatenate(segs)
    d = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).cuda()[: data.size]
    r = eng.validate(d, offs, F)
    f = r.batches["flags"]
    ok = int(np.sum((f & abi.F_CODEC_OK) != 0))
    dec = int(np.sum(r.batches["decoded_len"].astype(np.int64)[(f & abi.F_CODEC_OK) != 0]))
    out = eng.alloc_outputs(nseg, len(r.batches) + 16, int(r.totals["n_records"]) + 16, dec * 2 + (1 << 20))
    eng.set_timing(True)
    for _ in range(3):
        eng.submit(d, offs, out, F)
    torch.cuda.synchronize()
    tm = eng.last_timings()
    eng.set_timing(False)
    print(f"{'gzip' if codec == 1 else 'zstd'} {nseg}x{seg_mib}MiB batches {len(f)} ok {ok} decoded {dec/1e6:.1f} MB: plan+resolve {tm['resolve_plan']:.2f} ms "
          f"decode {tm['decode']:.2f} ms -> {dec / (tm['decode'] * 1e-3) / 1e9:.2f} GB/s decode pass", flush=True)
