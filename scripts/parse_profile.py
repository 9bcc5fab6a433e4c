"""Summarise a gpu_profile.sh run into profiles/<tag>_*: the kernel-trace stats
(copied) and the per-launch HBM traffic of k_validate from the PMC passes.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes
of a wide coalesced stream (the window loads are 16 B/lane dwordx4), so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Both are in KiB."""
import csv
import glob
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = os.path.join(root, "gpurun_out")
prof = os.path.join(root, "profiles")


def one(pattern):
    f = glob.glob(os.path.join(out, pattern), recursive=True)
    return f[0] if f else None


stats = one(f"prof_{tag}/**/*kernel_stats.csv")
if stats:
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))


def pmc(sub, name, kernel="k_validate"):
    f = one(f"{sub}/**/*counter_collection.csv")
    vals = []
    if not f:
        return None
    for row in csv.DictReader(open(f)):
        kn = row.get("Kernel_Name", "")
        if (kernel + "(") in kn.replace(" ", "") or kn.split("(")[0].strip().endswith(kernel):
            if row.get("Counter_Name") != name:
                continue
            vals.append(float(row["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None


fetch = pmc(f"pmc_fetch_{tag}", "FETCH_SIZE")
write = pmc(f"pmc_write_{tag}", "WRITE_SIZE")
fetch_np = pmc(f"pmc_fetchnp_{tag}", "FETCH_SIZE")  # CRC-only run (calibration), when collected
res = {"tag": tag, "kernel": "k_validate", "alg_def": "payload+128B/batch", "fetch_size_kib": fetch, "write_size_kib": write,
       "fetch_size_kib_crc_only": fetch_np,
       "correction": "FETCH_SIZE x2 (gfx950 counts half of a wide coalesced read; calibrated on the CRC-only run, "
                     "whose traffic is the dwordx4 window stream alone), WRITE_SIZE x1; KiB -> bytes"}
if fetch is not None and write is not None:
    res["bytes_per_launch"] = int(fetch * 1024 * 2 + write * 1024)
# the record walk (k_walk: per-lane 16-byte loads, so the x2 wide-stream
# correction is not calibrated for it: raw counter bytes are reported)
wf, ww = pmc(f"pmc_fetch_{tag}", "FETCH_SIZE", "k_walk"), pmc(f"pmc_write_{tag}", "WRITE_SIZE", "k_walk")
if wf is not None:
    res["walk"] = {"kernel": "k_walk", "fetch_size_kib": wf, "write_size_kib": ww,
                   "note": "raw FETCH_SIZE/WRITE_SIZE (uncalibrated for per-lane scattered 16-B loads)"}
for name in (f"{tag}_validate_traffic.json", "validate_traffic.json"):
    json.dump(res, open(os.path.join(prof, name), "w"), indent=1)
print(json.dumps(res))
