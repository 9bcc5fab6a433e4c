"""profiles/kernel_trace.json from a rocprofv3 --kernel-trace CSV of the
driver's exact bench command (bench.py --gpus 1 --steps S --warmup W):

    python scripts/trace_summary.py TAG gpurun_out/prof_TAG/TAG_kernel_trace.csv S W

C1 runs first in bench.py: its k_validate / k_walk launches are the first
W + S of each kernel (warm-up, then the S timed steps); the summary keeps the
mean of the S timed launches, which is what the bench line's HIP-event
kernel_ms averages over.  bench.py cites this file in roofline.trace."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C1_KERNELS = ("k_validate", "k_walk", "k_discover", "k_emit", "k_resolve", "k_chain", "k_finalize_bitmap")


def main():
    tag, path, steps, warmup = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    calls = {}
    for x in csv.DictReader(open(path)):
        n = x["Kernel_Name"].split("(")[0].replace("rp::", "").strip()
        calls.setdefault(n, []).append((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6)
    c1 = {}
    for k in C1_KERNELS:
        v = calls.get(k, [])
        if len(v) < warmup + steps:
            continue
        timed = v[warmup:warmup + steps]
        c1[k] = {"calls": len(timed), "mean_ms": round(sum(timed) / len(timed), 4),
                 "min_ms": round(min(timed), 4), "max_ms": round(max(timed), 4)}
    out = {"tag": tag, "command": f"rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps {steps} "
                                  f"--warmup {warmup}",
           "note": "C1's timed launches (the first warmup + steps launches of each kernel are C1's)", "c1": c1}
    with open(os.path.join(ROOT, "profiles", "kernel_trace.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
