# zstd / gzip member timings on one card: the zstd GPU tests, a job of eight
# 1 MiB members (scripts/mb_member_time.py), the RPGPU_ZSTAMPS variant's
# phase stamps (build it first: python scripts/build_exp.py zst --unit
# rp_inflate.hip -DRPGPU_ZSTAMPS), and a kernel trace of the member job.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-zm}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "zstd or codec or c6 or members or diag" > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 120 python scripts/mb_member_time.py zstd 3
timeout -k 10 120 python scripts/mb_member_time.py gzip 3
if [ -f redpanda_amd/librpgpu_zst.so ]; then
RPGPU_VARIANT=zst timeout -k 10 120 python -u scripts/mb_member_time.py zstd 1 > gpurun_out/zst_$TAG.out 2>&1 || { tail -30 gpurun_out/zst_$TAG.out; exit 1; }
grep -E "lane-parse|^zstd" gpurun_out/zst_$TAG.out | tail -3
fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o $TAG --output-format csv -- python3 scripts/mb_member_time.py zstd 2 > gpurun_out/prof_$TAG.log 2>&1
python - gpurun_out/prof_$TAG <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if float(r["TotalDurationNs"]) > 1e5:
        print(r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms avg")
PY
