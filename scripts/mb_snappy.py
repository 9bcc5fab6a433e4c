"""Microbenchmark (diagnostic): one segment holding a single ~1 MiB raw snappy
batch, validated + decoded 5 times; prints the decode stage (ms) — the
window-parallel walk of one long stream and its execution, in series."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import synth  # noqa: E402
from redpanda_amd import abi  # noqa: E402
from redpanda_amd.engine import Engine  # noqa: E402
import torch  # noqa: E402

a = np.zeros(1200 << 10, dtype=np.uint8)
n = synth.gen_segment(a, 0, seed=0x51, batch_bytes=0, min_batch=1 << 20, max_batch=1 << 20,
                      weights=[0, 0, 0, 0, 0, 1])
e = Engine(0)
e.set_timing(True)
d = torch.from_numpy(a).cuda()
offs = np.array([0, a.size], dtype=np.uint64)
flags = abi.JOB_CRC | abi.JOB_PARSE | abi.JOB_DECODE
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    r = e.validate(d, offs, flags, decoded_capacity=8 << 20)
    t = e.last_timings()
    print(f"batches {len(r.batches)} codec_ok {int(np.sum((r.batches['flags'] & abi.F_CODEC_OK) != 0))} "
          f"decode {t['decode']:.3f} ms total {t['total']:.3f} ms", flush=True)
