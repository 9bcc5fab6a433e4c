set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "zstd or codec or c6 or members or diag" > gpurun_out/pytest_r04r.log 2>&1 || { tail -60 gpurun_out/pytest_r04r.log; exit 1; }
tail -2 gpurun_out/pytest_r04r.log
timeout -k 10 120 python scripts/mb_member_time.py zstd 3
RPGPU_VARIANT=zst timeout -k 10 120 python -u scripts/mb_member_time.py zstd 1 > gpurun_out/zst_r04r.out 2>&1 || { tail -30 gpurun_out/zst_r04r.out; exit 1; }
grep -E "lane-parse|^zstd" gpurun_out/zst_r04r.out | tail -3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04r -o r04r --output-format csv -- python3 scripts/mb_member_time.py zstd 2 > gpurun_out/prof_r04r.log 2>&1
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_r04r/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if float(r["TotalDurationNs"]) > 1e5:
        print(r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms avg")
PY
