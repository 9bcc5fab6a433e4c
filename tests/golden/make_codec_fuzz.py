"""Writes the committed LZ4F / snappy mutation corpus:
tests/golden/codec_fuzz/frames.bin (the frames, concatenated) and
tests/golden/codec_fuzz/index.json (per frame: codec, kind, offset, length,
and the reference libraries' verdict: rc 0 / -1, decoded length and sha256).

Expected values come from liblz4 1.9.3 / libsnappy 1.1.8 through
oracle/_ref/libcodecref.so (built by oracle/Makefile in this container), the
drivers restating lz4_frame_compressor.cc:115-200 and
snappy_java_compressor.cc:76-129 / snappy_standard_compressor.cc:43-65.
Frames whose output exceeds the fixture capacity (rc -2) are left out.

    python tests/golden/make_codec_fuzz.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import codec_fuzz as F  # noqa: E402
from oracle import oracle as O  # noqa: E402

SEED = 0xF022
N_BASE, PER_BASE = 64, 9


def main():
    O.build()
    R = O.ref()
    assert R is not None, "oracle/_ref/libcodecref.so (liblz4 / libsnappy harness) is not built"
    frames = bytearray()
    index = []
    for codec, kind, f in F.corpus(R, SEED, N_BASE, PER_BASE):
        rc, out = F.ref_uncompress(R, codec, kind, f, F.cap_for(f))
        if rc == -2:
            continue
        index.append({"codec": codec, "kind": kind, "off": len(frames), "len": len(f), "rc": 0 if rc == 0 else -1,
                      "out_len": len(out), "out_sha256": hashlib.sha256(out).hexdigest()})
        frames += f
    d = os.path.join(HERE, "codec_fuzz")
    os.makedirs(d, exist_ok=True)
    open(os.path.join(d, "frames.bin"), "wb").write(bytes(frames))
    json.dump({"seed": SEED, "libraries": "liblz4 1.9.3, libsnappy 1.1.8 (oracle/_ref/libcodecref.so)",
               "frames": index}, open(os.path.join(d, "index.json"), "w"), indent=0)
    ok = sum(1 for e in index if e["rc"] == 0)
    print(f"{len(index)} frames ({ok} accepted), {len(frames)} bytes")


if __name__ == "__main__":
    main()
