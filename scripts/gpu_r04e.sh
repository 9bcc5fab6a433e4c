set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_check.sh r04e "" c1
RPGPU_VARIANT=pair timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_pair.log 2>&1 || { tail -40 gpurun_out/pytest_pair.log; exit 1; }
tail -2 gpurun_out/pytest_pair.log
bash scripts/gpu_ab.sh walk prev cur pair cur pair
