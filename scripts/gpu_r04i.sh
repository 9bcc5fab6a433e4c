# zstd lane parse: phase stamps, fast path on / off, kernel trace
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
RPGPU_VARIANT=zst timeout -k 10 120 python -u scripts/mb_member_time.py zstd 1 > gpurun_out/zst_r04i.out 2>&1 || { tail -30 gpurun_out/zst_r04i.out; exit 1; }
grep -E "ZSTAMPS|^zstd" gpurun_out/zst_r04i.out | tail -6
RPGPU_VARIANT=diag RPGPU_ZS_FAST=0 timeout -k 10 120 python scripts/mb_member_time.py zstd 3
RPGPU_VARIANT=diag timeout -k 10 120 python scripts/mb_member_time.py zstd 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04i -o r04i --output-format csv -- python3 scripts/mb_member_time.py zstd 2 > gpurun_out/prof_r04i.log 2>&1
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_r04i/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if float(r["TotalDurationNs"]) > 1e5:
        print(r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms avg")
PY
