# decoded record walk in its own LDS-free kernel (k_walk_decoded): GPU suite,
# then A/B: wvold (walk inside k_validate_decoded), wv5 (no occupancy hint)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r04o.log 2>&1 || { tail -60 gpurun_out/pytest_r04o.log; exit 1; }
tail -2 gpurun_out/pytest_r04o.log
W=c2,c5 bash scripts/gpu_ab.sh r04o cur wvold wv5 cur wvold wv5
