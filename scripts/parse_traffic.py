"""Per-kernel HBM traffic of one workload from rocprofv3 PMC passes
(scripts/gpu_traffic.sh) -> profiles/validate_traffic.json (c1) and
profiles/decode_traffic.json (c2, c5), plus a per-tag copy.

Counters (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE in KiB per
dispatch.  gfx950 correction: FETCH_SIZE x2 (it counts half of a wide
coalesced read; calibrated for 16-B-per-lane streams, which is how every
bulk reader here loads: k_validate's window rows, k_discover's scan rows,
k_lz_walk's staging rows, k_validate_decoded's rows); WRITE_SIZE x1.  Other
access widths are uncalibrated: the raw counters are kept beside the
corrected bytes.

Bytes are per submit: a kernel's counter summed over all its dispatches,
divided by the number of k_chunk_base dispatches (one per submit).
Algorithmic bytes per kernel come from the bench's --stats-out sidecar
(SURVEY §8(d) per-unit figures x the job's units)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(root, "gpurun_out")
prof = os.path.join(root, "profiles")


def counters(sub, name):
    files = glob.glob(os.path.join(out, sub, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(float)
    n = defaultdict(int)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != name:
                continue
            k = row.get("Kernel_Name", "").split("(")[0].replace("rp::", "").strip()
            k = k.split(" ")[-1].split("<")[0]
            acc[k] += float(row["Counter_Value"])
            n[k] += 1
    return acc, n


def alg_bytes(w, st):
    """Algorithmic bytes per submit, per kernel (None = no fixed figure)."""
    if not st:
        return {}
    sys.path.insert(0, root)
    from redpanda_amd import abi
    idx = abi.RECORD_INDEX.itemsize  # index entry bytes the walks write
    a = {
        # CRC of every stored payload, 128 B per batch result (read + write)
        "k_validate": st["stored_payload"] + 128 * st["batches"],
        "k_lz_walk": None,  # (round 5: only the pieces k_lzf_walk does not take)
        "k_validate_decoded": st["decoded"] + idx * st["records"],
    }
    z = st.get("lz4")
    if z:
        # round 6: the LZ4 kernels priced at their own
        # share.  k_raw_copy: stored blocks read + written; k_lzf_walk: the
        # compressed blocks read + 8 B records written; k_lz_exec: records +
        # literal bytes read (compressed bytes less >= 3 bytes of token /
        # offset per sequence) + the compressed blocks' output written
        seq = z["sequences_est"]
        a["k_raw_copy"] = 2 * z["raw_block_bytes"]
        a["k_lzf_walk"] = z["comp_block_bytes"] + 8 * seq
        a["k_lz_exec"] = 8 * seq + max(0, z["comp_block_bytes"] - 3 * seq) + z["comp_block_decoded"]
    else:
        a["k_lzf_walk"] = st["compressed_in"]
        a["k_lz_exec"] = st["decoded"]
    if w == "c1":
        a["k_walk"] = idx * st["records"] + 128 * st["batches"]
    return a


def one(tag, w):
    f, nf = counters(f"pmc_fetch_{tag}_{w}", "FETCH_SIZE")
    wr, nw = counters(f"pmc_write_{tag}_{w}", "WRITE_SIZE")
    subs = max(nf.get("k_chunk_base", 0), 1)
    subs_w = max(nw.get("k_chunk_base", 0), 1)
    try:
        st = json.load(open(os.path.join(out, f"stats_{tag}_{w}.json"))).get(w)
    except Exception:
        st = None
    alg = alg_bytes(w, st)
    ks = {}
    for k in sorted(set(f) | set(wr)):
        if not k.startswith("k_"):
            continue
        fk = f.get(k, 0.0) / subs
        wk = wr.get(k, 0.0) / subs_w
        b = int(fk * 1024 * 2 + wk * 1024)
        e = {"fetch_kib": round(fk, 1), "write_kib": round(wk, 1), "bytes": b}
        if k in alg and alg[k]:
            e["alg"] = int(alg[k])
            e["ratio"] = round(b / alg[k], 3)
        ks[k] = e
    return {"tag": tag, "submits_profiled": subs, "stats": st, "kernels": ks,
            "correction": "bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B), per submit; gfx950 FETCH_SIZE counts half "
                          "of a 16-B-per-lane coalesced stream (MI355X_MICROARCH.md §HBM)"}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r03"
    res = {w: one(tag, w) for w in ("c1", "c2", "c5", "c6")
           if os.path.isdir(os.path.join(out, f"pmc_fetch_{tag}_{w}"))}
    for w, r in res.items():
        print(w, json.dumps({k: (v["bytes"], v.get("ratio")) for k, v in r["kernels"].items()}))
    if "c1" in res:
        json.dump({"c1": res["c1"]}, open(os.path.join(prof, "validate_traffic.json"), "w"), indent=1)
    dec = {w: res[w] for w in ("c2", "c5", "c6") if w in res}
    if dec:
        json.dump(dec, open(os.path.join(prof, "decode_traffic.json"), "w"), indent=1)
    json.dump(res, open(os.path.join(prof, f"{tag}_traffic.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
