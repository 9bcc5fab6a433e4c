"""Write-side compressor throughput (diagnostic): rpgpu_compress_batch over
~256 MiB of mixed payloads (text / JSON / near-random, 64 KiB .. 1 MiB),
lz4 and snappy-java; wall time per call (host staging included) — the
kernel times come from a rocprofv3 kernel trace of the same run."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import compress_corpus as CC  # noqa: E402
from redpanda_amd.engine import Engine  # noqa: E402

rng = np.random.default_rng(1)
makers = [CC.text, CC.json_like, CC.mostly_random]
pays = []
tot = 0
while tot < (int(os.environ.get("MIB", "256")) << 20):
    n = int(rng.integers(65536, 1 << 20))
    pays.append(makers[len(pays) % 3](n, len(pays)))
    tot += n
e = Engine(0)
for codec in (3, 2):
    codecs = [codec] * len(pays)
    e.compress_batch(codecs[:4], pays[:4])
    t = time.perf_counter()
    res = e.compress_batch(codecs, pays)
    dt = time.perf_counter() - t
    out = sum(len(b) for _, b in res)
    assert all(s == 0 for s, _ in res)
    print(f"codec {codec}: {len(pays)} payloads {tot / 2**20:.0f} MiB -> {out / 2**20:.0f} MiB in {dt * 1e3:.1f} ms "
          f"({tot / dt / 1e9:.2f} GB/s incl. host staging)", flush=True)
