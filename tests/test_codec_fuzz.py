"""LZ4F / snappy mutation parity.

* test_oracle_matches_libraries: the oracle's restatement
  (oracle/rp_oracle.c rpo_lz4f_uncompress / rpo_snappy_*_uncompress) against
  liblz4 1.9.3 / libsnappy 1.1.8 themselves (oracle/_ref/libcodecref.so) on
  ~12 K seeded mutations of library-made frames (tests/codec_fuzz.py):
  accept / reject and decoded bytes identical.
* test_oracle_matches_committed_corpus: the same for the committed corpus
  (tests/golden/codec_fuzz, made by tests/golden/make_codec_fuzz.py from the
  libraries), which needs no library at run time.
* test_gpu_corpus_job / test_gpu_corpus_uncompress_batch (-m gpu): the
  committed corpus through the HIP job pipeline (one batch per frame, field by
  field against the oracle, and each accepted frame's decoded bytes against
  the libraries' sha256) and through rpgpu_uncompress_batch.
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

from redpanda_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import batchgen as bg  # noqa: E402
import codec_fuzz as F  # noqa: E402

G = os.path.join(HERE, "golden", "codec_fuzz")
JFLAGS = abi.JOB_CRC | abi.JOB_PARSE | abi.JOB_DECODE


def _corpus():
    idx = json.load(open(os.path.join(G, "index.json")))["frames"]
    blob = open(os.path.join(G, "frames.bin"), "rb").read()
    return [(e, blob[e["off"]: e["off"] + e["len"]]) for e in idx]


@pytest.mark.parametrize("seed,max_in", [(1, 6000), (2, 6000), (3, 200000)])
def test_oracle_matches_libraries(oracle, seed, max_in):
    R = oracle.ref()
    if R is None:
        pytest.skip("oracle/_ref/libcodecref.so (liblz4 / libsnappy) not built")
    n_base = 300 if max_in <= 6000 else 40
    cor = F.corpus(R, 0xF000 + seed, n_base, 12, max_in=max_in)
    bad, acc = [], 0
    for codec, kind, f in cor:
        cap = F.cap_for(f)
        rr, rb = F.ref_uncompress(R, codec, kind, f, cap)
        orc, ob = oracle.uncompress(codec, f, cap)
        acc += rr == 0
        if rr != orc or rb != ob:
            bad.append((kind, rr, orc, len(f), f[:32].hex()))
    assert not bad, bad[:5]
    assert len(cor) >= 3000 or max_in > 6000
    assert 0.1 * len(cor) < acc < 0.9 * len(cor)


def test_oracle_matches_committed_corpus(oracle):
    cor = _corpus()
    assert len(cor) >= 500
    assert {e["kind"] for e, _ in cor} == {"lz4f", "raw", "java"}
    for e, f in cor:
        rc, out = oracle.uncompress(e["codec"], f, F.cap_for(f))
        assert (0 if rc == 0 else -1) == e["rc"], e
        assert len(out) == e["out_len"] and hashlib.sha256(out).hexdigest() == e["out_sha256"], e


def corpus_segments():
    """The corpus as batches (one frame each, its codec in attrs), two segments."""
    cor = _corpus()
    segs = []
    for part in (cor[0::2], cor[1::2]):
        out = bytearray()
        for i, (e, f) in enumerate(part):
            out += bg.batch(f, 1, base_offset=i, attrs=e["codec"])
        segs.append(np.frombuffer(bytes(out), dtype=np.uint8).copy())
    return segs, [cor[0::2], cor[1::2]]


def _job_vs_libraries(res, parts):
    """Per batch: a frame the libraries reject is never decoded; an accepted
    one decodes to the libraries' bytes unless the job's decode capacity (the
    frame plan rule) refused it.  Returns the accepted frames decoded."""
    b = res.batches
    k = decoded = 0
    for part in parts:
        for e, f in part:
            fl = int(b["flags"][k])
            if e["rc"] != 0:
                assert not fl & abi.F_CODEC_OK, (k, e)
            elif fl & abi.F_CODEC_OK:
                o, n = int(b["decoded_off"][k]), int(b["decoded_len"][k])
                assert n == e["out_len"] and hashlib.sha256(bytes(res.decoded[o:o + n])).hexdigest() == e["out_sha256"]
                decoded += 1
            k += 1
    assert k == len(b)
    return decoded


def test_oracle_job_on_corpus(oracle):
    """The oracle's whole-job run (the GPU test's checker) agrees with the
    libraries on the corpus."""
    segs, parts = corpus_segments()
    offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
    data = np.concatenate(segs)
    ref = oracle.run_job(data, offs, JFLAGS, decoded_cap=data.size * 64)
    n_ok = sum(1 for p in parts for e, _ in p if e["rc"] == 0)
    assert _job_vs_libraries(ref, parts) >= n_ok - 8


@pytest.mark.gpu
def test_gpu_corpus_job(engine, oracle):
    import torch
    from test_gpu_parity import assert_same
    segs, parts = corpus_segments()
    offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
    data = np.concatenate(segs)
    # one decode-arena capacity for both: mutated frames claim large plans
    # (content sizes, block maxima), and an arena that runs out sets the same
    # DECODE_OVERFLOW bits in both only when both have the same room
    cap = data.size * 64
    ref = oracle.run_job(data, offs, JFLAGS, decoded_cap=cap)
    d = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).cuda()[: data.size]
    got = engine.validate(d, offs, JFLAGS, decoded_capacity=cap)
    assert_same(got, ref, JFLAGS)
    n_ok = sum(1 for p in parts for e, _ in p if e["rc"] == 0)
    assert _job_vs_libraries(got, parts) >= n_ok - 8


@pytest.mark.gpu
def test_gpu_corpus_uncompress_batch(engine):
    cor = _corpus()
    res = engine.uncompress_batch([e["codec"] for e, _ in cor], [f for _, f in cor],
                                  caps=[F.cap_for(f) for _, f in cor])
    for (e, f), (st, got) in zip(cor, res):
        if e["rc"] == 0:
            assert st == 0 and len(got) == e["out_len"] and hashlib.sha256(got).hexdigest() == e["out_sha256"], e
        else:
            assert st == abi.E_CODEC, (e, st)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12])
def test_gpu_fuzz_job(engine, oracle, seed):
    """~5,200 fresh mutations per seed (library-made frames, tests/codec_fuzz.py)
    through one HIP job, field by field against the oracle's job; the
    oracle is pinned to the libraries by test_oracle_matches_libraries."""
    import torch
    from test_gpu_parity import assert_same
    R = oracle.ref()
    if R is None:
        pytest.skip("oracle/_ref/libcodecref.so not built")
    cor = F.corpus(R, 0xF100 + seed, 400, 12)
    segs = []
    for part in (cor[0::2], cor[1::2]):
        out = bytearray()
        for i, (codec, _kind, f) in enumerate(part):
            out += bg.batch(f, 1, base_offset=i, attrs=codec)
        segs.append(np.frombuffer(bytes(out), dtype=np.uint8).copy())
    offs = np.cumsum([0] + [s.size for s in segs]).astype(np.uint64)
    data = np.concatenate(segs)
    cap = data.size * 64
    ref = oracle.run_job(data, offs, JFLAGS, decoded_cap=cap)
    d = torch.from_numpy(np.concatenate([data, np.zeros(16, np.uint8)])).cuda()[: data.size]
    got = engine.validate(d, offs, JFLAGS, decoded_capacity=cap)
    ok = (ref.batches["flags"] & abi.F_CODEC_OK) != 0
    assert len(ref.batches) == len(cor) and 0.1 * len(cor) < int(np.sum(ok)) < 0.9 * len(cor)
    assert_same(got, ref, JFLAGS)
