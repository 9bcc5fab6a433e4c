set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
RPGPU_VARIANT=zuni timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "zstd" > gpurun_out/pytest_r04s.log 2>&1 || { tail -60 gpurun_out/pytest_r04s.log; exit 1; }
tail -2 gpurun_out/pytest_r04s.log
for V in cur zuni cur zuni; do
  if [ $V = cur ]; then unset RPGPU_VARIANT; else export RPGPU_VARIANT=$V; fi
  timeout -k 10 120 python scripts/mb_member_time.py zstd 3
done
