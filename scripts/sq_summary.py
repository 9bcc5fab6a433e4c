"""Print k_validate's SQ counters (summed over dimensions) from a gpu_sq.sh run."""
import csv, glob, sys, collections
tag = sys.argv[1] if len(sys.argv) > 1 else "sq"
kern = sys.argv[2] if len(sys.argv) > 2 else "k_validate"
vals = collections.defaultdict(float)
for f in glob.glob(f"gpurun_out/{tag}_*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            vals[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(vals):
    print(f"{k:24s} {vals[k]:.4g}")
