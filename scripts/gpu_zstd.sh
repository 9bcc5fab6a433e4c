# zstd on the device (rp_zstd_core.h via rp_inflate.hip): zstd + gzip job parity, then the C6 stanza
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "zstd or gzip" > gpurun_out/pytest_zstd.log 2>&1 || { tail -60 gpurun_out/pytest_zstd.log; exit 1; }
tail -12 gpurun_out/pytest_zstd.log
