"""Golden vectors of the write side's compressors: sha256 + length of what
liblz4 1.9.3 / libsnappy 1.1.8 produce through the reference's wrapper loops
(oracle/_ref/libcodecref.so: ref_lz4f_compress_stream = lz4_frame_compressor
::compress, ref_snappy_java_compress = snappy_java_compressor::compress) on
tests/compress_corpus.py's payloads.  They pin the oracle's restatement where
the harness cannot be built.  Run: python tests/golden/make_compress_golden.py"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import compress_corpus  # noqa: E402
from oracle import oracle  # noqa: E402

out = {}
for name, data in compress_corpus.cases():
    for codec, cname in ((3, "lz4"), (2, "snappy")):
        for frag in (compress_corpus.FRAGS if codec == 2 else (0,)):
            r = oracle.ref_compress(codec, data, frag)
            assert r is not None, "oracle/_ref harness not built"
            out[f"{cname}/{name}/{frag}"] = [len(r), hashlib.sha256(r).hexdigest()]
with open(os.path.join(HERE, "compress_vectors.json"), "w") as f:
    json.dump(out, f, indent=0, sort_keys=True)
print(len(out), "vectors")
