# 8 KiB exec ring (16 waves per CU) vs the 16 KiB ring: decode parity on the
# variant, then C2/C5 interleaved.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
RPGPU_VARIANT=ring8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_ring8.log 2>&1 || { tail -40 gpurun_out/pytest_ring8.log; exit 1; }
tail -2 gpurun_out/pytest_ring8.log
W=c2,c5 bash scripts/gpu_ab.sh r04g cur ring8 cur ring8
