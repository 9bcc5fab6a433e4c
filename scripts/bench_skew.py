"""Skewed-job diagnostic for the split CRC (k_crc_split / k_crc_combine): a
job of 64 stored batches of 2..4 MiB (one segment) validated with the
default split threshold and with splitting off (RPGPU_SPLIT_MIN_KIB in a
child process); prints ms per submit for each."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    import synth
    from redpanda_amd import abi
    from redpanda_amd.engine import Engine
    a = np.zeros(200 << 20, dtype=np.uint8)
    synth.gen_segment(a, 0, seed=0x5E, batch_bytes=0, min_batch=2 << 20, max_batch=4 << 20)
    e = Engine(0)
    d = torch.from_numpy(a).cuda()
    offs = np.array([0, a.size], dtype=np.uint64)
    for _ in range(3):
        r = e.validate(d, offs, abi.JOB_CRC)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        r = e.validate(d, offs, abi.JOB_CRC)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 100
    ok = int(np.sum((r.batches["flags"] & abi.F_CRC_OK) != 0))
    print(json.dumps({"ms": round(ms, 3), "batches": len(r.batches), "crc_ok": ok}))
    sys.exit(0)
for label, env in (("split", {}), ("no-split", {"RPGPU_SPLIT_MIN_KIB": str(1 << 30)})):
    out = subprocess.run([sys.executable, __file__, "child"], env={**os.environ, **env}, capture_output=True,
                         text=True, timeout=300)
    print(label, out.stdout.strip() or out.stderr[-500:], flush=True)
