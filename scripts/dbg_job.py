"""Debug: one C2/C5 recipe job through rpgpu_submit with RPGPU_DEBUG_SYNC=1
(each stage synchronised and named on stderr), in a bounded subprocess;
compares with the oracle.  Usage: dbg_job.py [c2|c5] [nseg] [seg_mib]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import synth
    from oracle import oracle as O
    from redpanda_amd import abi
    import torch
    from redpanda_amd.engine import Engine
    which = sys.argv[1] if len(sys.argv) > 1 else "c2"
    nseg = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    mib = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    kw = dict(synth.C2, lz4_linked_ppm=300000, lz4_content_checksum_ppm=300000,
              lz4_block_checksum_ppm=100000) if which == "c2" else synth.C5
    segs = []
    for i in range(nseg):
        a = np.zeros(mib << 20, np.uint8)
        synth.gen_segment(a, i, **kw)
        segs.append(a)
    offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
    data = np.concatenate(segs)
    flags = abi.JOB_CRC | abi.JOB_PARSE | abi.JOB_DECODE
    print("oracle...", flush=True)
    ref = O.run_job(data, offs, flags)
    print("gpu...", flush=True)
    e = Engine(0)
    d = torch.from_numpy(np.concatenate([data, np.zeros(256, np.uint8)])).cuda()
    got = e.validate(d, offs, flags, chunk_bytes=256 << 10)
    print("compare", flush=True)
    bad = [f for f in abi.BATCH_COMPARE_FIELDS if not np.array_equal(got.batches[f], ref.batches[f])]
    print("batches", len(got.batches), len(ref.batches), "bad fields", bad, flush=True)
    if bad:
        for f in bad[:3]:
            idx = np.nonzero(got.batches[f] != ref.batches[f])[0]
            print(f, idx[:10], got.batches[f][idx[:5]], ref.batches[f][idx[:5]], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
