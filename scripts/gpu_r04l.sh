# ZLane uniform (SGPR) state vs VGPR state: zstd GPU parity, member timings
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "zstd or codec or c6 or members" > gpurun_out/pytest_r04l.log 2>&1 || { tail -60 gpurun_out/pytest_r04l.log; exit 1; }
tail -2 gpurun_out/pytest_r04l.log
for V in cur zlv cur zlv; do
  if [ $V = cur ]; then unset RPGPU_VARIANT; else export RPGPU_VARIANT=$V; fi
  timeout -k 10 120 python scripts/mb_member_time.py zstd 3
done
unset RPGPU_VARIANT
RPGPU_VARIANT=zst timeout -k 10 120 python -u scripts/mb_member_time.py zstd 1 > gpurun_out/zst_r04l.out 2>&1 || { tail -30 gpurun_out/zst_r04l.out; exit 1; }
grep -E "lane-parse|^zstd" gpurun_out/zst_r04l.out | tail -3
