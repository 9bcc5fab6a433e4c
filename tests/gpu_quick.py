"""Quick end-to-end GPU check (development helper, not collected by pytest)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from redpanda_amd import _lib, abi
from redpanda_amd.engine import Engine
from oracle import oracle as O
import synth  # noqa: E402  (test/bench data generator, not the product)

def cmp(name, a, b, fields):
    ok = True
    if len(a) != len(b):
        print(name, "LEN MISMATCH", len(a), len(b)); return False
    for f in fields:
        if not np.array_equal(a[f], b[f]):
            idx = np.nonzero(a[f] != b[f])[0]
            print(name, "field", f, "mismatch at", idx[:5], a[f][idx[:5]], b[f][idx[:5]]); ok = False
    return ok

e = Engine(0)
for case in range(4):
    seg_bytes = [4 << 20, 1 << 20, 3 << 20 | 12345]
    segs = []
    for i, sb in enumerate(seg_bytes):
        a = np.zeros(sb, dtype=np.uint8)
        if case == 0:
            synth.gen_segment(a, i, seed=1)
        elif case == 1:
            synth.gen_segment(a, i, seed=2, batch_bytes=0, min_batch=200, max_batch=200000)
        elif case == 2:
            synth.gen_segment(a, i, seed=3, batch_bytes=0, min_batch=200, max_batch=100000, corrupt_payload_ppm=50000, value_bytes=100)
        else:
            synth.gen_segment(a, i, seed=4, batch_bytes=0, min_batch=200, max_batch=600000, corrupt_payload_ppm=10000, corrupt_header_ppm=5000)
        segs.append(a)
    offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
    data = np.concatenate(segs)
    flags = abi.JOB_CRC | abi.JOB_PARSE
    ref = O.run_job(data, offs, flags)
    d = torch.from_numpy(data).cuda()
    for cb in (0, 65536, 4096):
        t = time.time()
        got = e.validate(d, offs, flags, chunk_bytes=cb)
        ok = cmp(f"case{case} cb{cb} batches", got.batches, ref.batches, abi.BATCH_COMPARE_FIELDS)
        ok &= cmp(f"case{case} cb{cb} records", got.records, ref.records, abi.RECORD_COMPARE_FIELDS)
        ok &= cmp(f"case{case} cb{cb} summaries", got.summaries, ref.summaries, abi.SUMMARY_COMPARE_FIELDS)
        for k in ("n_batches", "n_records", "decoded_bytes"):
            if got.totals[k] != ref.totals[k]:
                print("totals", k, got.totals[k], ref.totals[k]); ok = False
        print(f"case{case} chunk={cb}: batches={len(got.batches)} records={len(got.records)} rewalks={got.totals['n_rewalks']} ok={ok} ({time.time()-t:.2f}s)")
print("DONE")
