# zstd lane parse with interleaved four-stream literals: zstd GPU parity,
# phase stamps, fast path on / off
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "zstd or gzip or c6 or members or codec" > gpurun_out/pytest_r04j.log 2>&1 || { tail -60 gpurun_out/pytest_r04j.log; exit 1; }
tail -2 gpurun_out/pytest_r04j.log
RPGPU_VARIANT=zst timeout -k 10 120 python -u scripts/mb_member_time.py zstd 1 > gpurun_out/zst_r04j.out 2>&1 || { tail -30 gpurun_out/zst_r04j.out; exit 1; }
grep -E "lane-parse|^zstd" gpurun_out/zst_r04j.out | tail -3
RPGPU_VARIANT=diag RPGPU_ZS_FAST=0 timeout -k 10 120 python scripts/mb_member_time.py zstd 3
timeout -k 10 120 python scripts/mb_member_time.py zstd 3
