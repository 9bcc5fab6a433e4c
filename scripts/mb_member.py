"""One job of 1 MiB gzip or zstd members (diagnostic, for counter passes):
python scripts/mb_member.py gzip|zstd [reps]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import synth
from redpanda_amd import abi
from redpanda_amd.engine import Engine

codec = {"gzip": 1, "zstd": 4}[sys.argv[1]]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
w = [0] * 6
w[codec] = 1
a = np.zeros(4 << 20, np.uint8)
synth.gen_segment(a, 0, seed=77, batch_bytes=0, min_batch=1 << 20, max_batch=1 << 20, weights=w, size_uniform=True)
offs = np.array([0, a.size], np.uint64)
d = torch.from_numpy(np.concatenate([a, np.zeros(16, np.uint8)])).cuda()[: a.size]
eng = Engine(0)
F = abi.JOB_CRC | abi.JOB_PARSE | abi.JOB_DECODE
r = eng.validate(d, offs, F)
for _ in range(reps):
    r = eng.validate(d, offs, F)
torch.cuda.synchronize()
f = r.batches["flags"]
print(sys.argv[1], "batches", len(f), "ok", int(np.sum((f & abi.F_CODEC_OK) != 0)))
