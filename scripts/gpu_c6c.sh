# gzip / zstd parity, then the C6 stanza with its CPU baseline
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "zstd or gzip" > gpurun_out/pytest_zstd.log 2>&1 || { tail -60 gpurun_out/pytest_zstd.log; exit 1; }
tail -2 gpurun_out/pytest_zstd.log
bash scripts/gpu_c6base.sh
