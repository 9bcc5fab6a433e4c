"""Debug: the committed LZ4F / snappy corpus (tests/golden/codec_fuzz) through
one HIP job and through rpgpu_uncompress, printing every frame whose verdict
or bytes differ from the oracle (and the libraries' fixture values)."""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import test_codec_fuzz as T
    from oracle import oracle as O
    from redpanda_amd import abi
    from redpanda_amd.engine import Engine
    O.build()
    eng = Engine(0)
    segs, parts = T.corpus_segments()
    offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
    data = np.concatenate(segs)
    cap = data.size * 64
    ref = O.run_job(data, offs, T.JFLAGS, decoded_cap=cap)
    d = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).cuda()[: data.size]
    got = eng.validate(d, offs, T.JFLAGS, decoded_capacity=cap)
    ents = [e for p in parts for e in p]
    bad = 0
    for k in range(len(ref.batches)):
        diffs = [f for f in abi.BATCH_COMPARE_FIELDS if got.batches[f][k] != ref.batches[f][k]]
        if not diffs:
            continue
        bad += 1
        e, f = ents[k]
        print("batch", k, "kind", e["kind"], "lib rc", e["rc"], "len", e["len"], "diff fields", diffs,
              {x: (int(got.batches[x][k]), int(ref.batches[x][k])) for x in diffs})
        try:
            g = eng.uncompress(e["codec"], f, max(len(f) * 300, 1 << 20))
            print("  rpgpu_uncompress: ok", len(g), hashlib.sha256(g).hexdigest() == e["out_sha256"])
        except Exception as ex:  # noqa: BLE001
            print("  rpgpu_uncompress: raised", ex)
        print("  frame", f.hex())
    print("mismatching batches:", bad)


if __name__ == "__main__":
    main()
