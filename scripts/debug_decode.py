"""Diagnostic: run the codec-mix parity input and report, per mismatching
batch, its codec, frame shape and the first differing decoded byte."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from oracle import oracle as O
    from redpanda_amd import _lib, abi
    from redpanda_amd.engine import Engine
    mix = (1 << abi.CODEC_NONE) | (1 << abi.CODEC_LZ4) | (1 << abi.CODEC_SNAPPY)
    segs = []
    for i in range(3):
        a = np.zeros(3 << 20, dtype=np.uint8)
        _lib.gen_segment(a, i, seed=0xC2, batch_bytes=0, min_batch=200, max_batch=700000, codec_mix=mix,
                         corrupt_payload_ppm=(20000 if i == 1 else 0))
        segs.append(a)
    offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
    data = np.concatenate(segs)
    flags = abi.JOB_CRC | abi.JOB_PARSE | abi.JOB_DECODE
    ref = O.run_job(data, offs, flags)
    eng = Engine(0)
    for rep in range(int(os.environ.get("REPS", "3"))):
        got = eng.validate(torch.from_numpy(data).cuda(), offs, flags, chunk_bytes=64 << 10)
        bad = np.nonzero(got.batches["flags"] != ref.batches["flags"])[0]
        print(f"rep {rep}: {len(bad)} flag mismatches", flush=True)
        for i in bad[:5]:
            b, r = got.batches[i], ref.batches[i]
            seg = int(b["segment"])
            p = int(offs[seg]) + int(b["file_pos"]) + 61
            n = int(b["size_bytes"]) - 61
            codec = int(b["attrs"]) & 7
            payload = data[p:p + n].tobytes()
            off, ln = int(r["decoded_off"]), int(r["decoded_len"])
            gd, rd = got.decoded[off:off + ln], ref.decoded[off:off + ln]
            diff = np.nonzero(gd != rd)[0]
            flg = payload[4] if codec == abi.CODEC_LZ4 else -1
            print(f"  batch {i}: codec {codec} n={n} flags got {int(b['flags']):#x} ref {int(r['flags']):#x} "
                  f"dlen got {int(b['decoded_len'])} ref {ln} lz4 flg={flg:#x} "
                  f"first diff {diff[0] if len(diff) else None} ndiff {len(diff)}", flush=True)


if __name__ == "__main__":
    main()
