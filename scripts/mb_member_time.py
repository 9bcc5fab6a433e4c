"""Wall time of one job of four 1 MiB gzip or zstd members (one wave per
member: the time of the member pass is one member's serial decode).
python scripts/mb_member_time.py gzip|zstd [reps]  (RPGPU_VARIANT picks the library)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import synth  # noqa: E402
from redpanda_amd import abi  # noqa: E402
from redpanda_amd.engine import Engine  # noqa: E402

name = sys.argv[1]
codec = {"gzip": 1, "zstd": 4}[name]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
w = [0] * 6
w[codec] = 1
a = np.zeros(4 << 20, np.uint8)
synth.gen_segment(a, 0, seed=77, batch_bytes=0, min_batch=1 << 20, max_batch=1 << 20, weights=w, size_uniform=True)
offs = np.array([0, a.size], np.uint64)
d = torch.from_numpy(np.concatenate([a, np.zeros(16, np.uint8)])).cuda()[: a.size]
eng = Engine(0)
F = abi.JOB_CRC | abi.JOB_PARSE | abi.JOB_DECODE
r = eng.validate(d, offs, F)
torch.cuda.synchronize()
t = []
for _ in range(reps):
    t0 = time.perf_counter()
    r = eng.validate(d, offs, F)
    torch.cuda.synchronize()
    t.append(time.perf_counter() - t0)
f = r.batches["flags"]
print(name, os.environ.get("RPGPU_VARIANT", "cur"), "batches", len(f), "ok", int(np.sum((f & abi.F_CODEC_OK) != 0)),
      "decoded", int(np.sum(r.batches["decoded_len"].astype(np.int64))), "ms", round(min(t) * 1e3, 2))
