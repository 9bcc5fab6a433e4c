set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_check.sh r04e "" c1
RPGPU_VARIANT=pair timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_pair.log 2>&1 || { tail -40 gpurun_out/pytest_pair.log; exit 1; }
tail -2 gpurun_out/pytest_pair.log
for V in prev cur; do
  if [ $V = cur ]; then unset RPGPU_VARIANT; else export RPGPU_VARIANT=$V; fi
  timeout -k 10 120 python scripts/mb_member_time.py gzip 3
  timeout -k 10 120 python scripts/mb_member_time.py zstd 3
done
unset RPGPU_VARIANT
bash scripts/gpu_ab.sh walk prev cur pair cur pair
