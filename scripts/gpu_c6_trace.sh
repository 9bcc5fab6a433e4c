# C6 kernel trace (member kernels) and the 1 MiB member timings on one card.
# Diagnostics only.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-c6t}
timeout -k 10 120 python scripts/mb_member_time.py gzip 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o $TAG --output-format csv -- python3 bench.py --workloads c6 --no-cpu-baseline --no-index --steps 2 --warmup 1 > gpurun_out/prof_$TAG.log 2>&1
python - gpurun_out/prof_$TAG <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if float(r["TotalDurationNs"]) > 1e6:
        print(r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms avg", round(float(r["MaxNs"]) / 1e6, 3), "max")
PY
