"""Diagnostic: gzip batches where the device and the oracle disagree
(payload size / alignment, block types, plan vs decode)."""
import sys, os, zlib
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import synth
from oracle import oracle as O
from redpanda_amd import abi
from redpanda_amd.engine import Engine
from tests.test_gpu_parity import GZ_WEIGHTS, DFLAGS

def blocks(p):
    d = p[10:]
    bit = 0
    out = []
    def bits(n):
        nonlocal bit
        v = 0
        for i in range(n):
            v |= ((d[bit >> 3] >> (bit & 7)) & 1) << i
            bit += 1
        return v
    try:
        last = bits(1); t = bits(2); out.append(t)
    except IndexError:
        pass
    return out

eng = Engine(0)
for seed in (198, 0xC6):
    segs = []
    for i in range(3):
        a = np.zeros(3 << 20, np.uint8)
        synth.gen_segment(a, i, seed=seed, batch_bytes=0, min_batch=200, max_batch=600000, weights=GZ_WEIGHTS,
                          corrupt_payload_ppm=(20000 if i == 1 else 0))
        segs.append(a)
    offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
    data = np.concatenate(segs)
    ref = O.run_job(data, offs, DFLAGS)
    d = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).cuda()[: data.size]
    got = eng.validate(d, offs, DFLAGS, chunk_bytes=64 << 10)
    gb, rb = got.batches, ref.batches
    for k in range(len(rb)):
        if gb["flags"][k] != rb["flags"][k]:
            S = int(offs[rb["segment"][k]]) + int(rb["file_pos"][k]) + 61
            n = int(rb["size_bytes"][k]) - 61
            p = data[S:S + n].tobytes()
            print(seed, k, "codec", rb["attrs"][k] & 7, "n", n, "mis", S & 3, "flags dev/ref", gb["flags"][k], rb["flags"][k],
                  "dlen dev/ref", gb["decoded_len"][k], rb["decoded_len"][k], "doff dev/ref", gb["decoded_off"][k],
                  rb["decoded_off"][k], "first block", blocks(p), "zlib", len(zlib.decompressobj(47).decompress(p)))
