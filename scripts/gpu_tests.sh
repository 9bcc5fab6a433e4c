# GPU parity tests only (optionally a -k filter); bounded, verbose log under gpurun_out/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-t}
K=${2:-}
if [ -n "$K" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1 || { tail -80 gpurun_out/pytest_$TAG.log; exit 1; }
else
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -80 gpurun_out/pytest_$TAG.log; exit 1; }
fi
tail -5 gpurun_out/pytest_$TAG.log
