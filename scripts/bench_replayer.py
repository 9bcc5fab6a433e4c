"""log_replayer::recover (the C++ drop-in surface, include/rpgpu_redpanda.h)
over host-resident 1 GiB C1 segments through the pinned, double-buffered
host path: the C++ driver times it (tests/cpp/surfaces_main.cpp
recover_bench).  Prints one JSON line.  Diagnostic beside bench.py."""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import synth  # noqa: E402  (test/bench data generator, not the product)
from redpanda_amd import build as B  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
drv = B.SURFACES_BIN
d = tempfile.mkdtemp(dir="/tmp")
paths = []
for p in range(n):
    a = np.zeros(1 << 30, np.uint8)
    synth.gen_segment(a, p, seed=0xC1)
    path = os.path.join(d, f"seg{p}.bin")
    a.tofile(path)
    paths.append(path)
    del a
try:
    r = subprocess.run([drv, "recover_bench", str(reps)] + paths, capture_output=True, text=True, timeout=600)
finally:
    for path in paths:
        os.unlink(path)
    os.rmdir(d)
line = [x for x in r.stdout.splitlines() if x.startswith("RECOVER_BENCH")]
if r.returncode != 0 or not line:
    sys.stderr.write(r.stdout + r.stderr)
    sys.exit(1)
kv = dict(x.split("=") for x in line[0].split()[1:])
print(json.dumps({"surface": "storage::log_replayer::recover", "segments": n, "segment_bytes": 1 << 30,
                  "reps": reps, "seconds": float(kv["seconds"]), "GBps": float(kv["GBps"]),
                  "path": "rpgpu_validate_host (pinned staging, 256 MiB groups, copy stream + compute stream)"}))
