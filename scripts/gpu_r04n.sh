# decoded payloads walked by k_walk lanes: GPU suite, then A/B against the
# wave walk (dww) on C2 / C5
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r04n.log 2>&1 || { tail -60 gpurun_out/pytest_r04n.log; exit 1; }
tail -2 gpurun_out/pytest_r04n.log
W=c2,c5 bash scripts/gpu_ab.sh r04n cur dww cur dww
