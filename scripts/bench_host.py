"""PCIe-inclusive rate of the host segment path (rpgpu_validate_host):
host-resident C1 segments (pinned with torch, or pageable with --pageable)
copied H2D in double-buffered staging groups and validated on the device.
Diagnostic beside bench.py (whose value is the device-resident rate)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from redpanda_amd import _lib, abi  # noqa: E402
from redpanda_amd.engine import Engine  # noqa: E402
import synth  # noqa: E402  (test/bench data generator, not the product)

ap = argparse.ArgumentParser()
ap.add_argument("--partitions", type=int, default=8)
ap.add_argument("--seg-gib", type=float, default=1.0)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--pageable", action="store_true")
ap.add_argument("--no-records", action="store_true", help="do not return the record index to the host")
a = ap.parse_args()
seg = int(a.seg_gib * (1 << 30)) // 16384 * 16384
segs = []
for p in range(a.partitions):
    t = torch.empty(seg, dtype=torch.uint8, pin_memory=not a.pageable)
    synth.gen_segment(t.numpy(), p, seed=0xC1)
    segs.append(t.numpy())
eng = Engine(0)
flags = abi.JOB_CRC | abi.JOB_PARSE
rcap = 0 if a.no_records else None
r = eng.validate_host(segs, flags, record_capacity=rcap)  # warm-up (allocates the staging slots)
b, tot = r.batches, r.totals
ok = bool(np.all(b["flags"] & abi.F_CRC_OK) and np.all(b["flags"] & abi.F_PARSE_OK)
          and (a.no_records or len(r.records) == int(tot["n_records"])))
times = []
for _ in range(a.reps):
    t0 = time.perf_counter()
    r = eng.validate_host(segs, flags, record_capacity=rcap)
    times.append(time.perf_counter() - t0)
tot = r.totals
best = min(times)
total = seg * a.partitions
print(json.dumps({"path": "rpgpu_validate_host", "pinned": not a.pageable, "bytes": total,
                  "records_returned": not a.no_records, "records": int(tot["n_records"]),
                  "batches": int(tot["n_batches"]), "all_valid": ok, "best_s": round(best, 4),
                  "GBps": round(total / best / 1e9, 1)}))
