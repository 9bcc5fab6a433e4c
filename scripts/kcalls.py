"""Per-call durations (ms) of the engine's kernels from a rocprofv3 kernel trace."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
names = {}
for x in rows:
    n = x["Kernel_Name"].split("(")[0].replace("rp::", "")
    if n.startswith("__amd") or n.startswith("void at::"):
        continue
    names.setdefault(n, []).append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6)
for n, v in sorted(names.items(), key=lambda kv: -sum(kv[1])):
    print(f"{n:24s} calls={len(v):3d} total={sum(v):9.3f} ms  per call: " + " ".join(f"{d:.3f}" for d in v[:12]))
