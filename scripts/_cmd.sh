set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -40 gpurun_out/pytest_iter.log; exit 1; }
tail -3 gpurun_out/pytest_iter.log
