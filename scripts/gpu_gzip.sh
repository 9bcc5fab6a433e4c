# gzip-in-job parity (rp_inflate.hip), the decode / wire / C++-surface tests
# around it; every GPU step bounded, chained with &&
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_surfaces.py -m gpu -x -v --timeout 200 \
  --timeout-method thread -k "gzip or codec_mix or decode_without or serialize_wire or index or uncompress" \
  > gpurun_out/pytest_gzip.log 2>&1 || { tail -60 gpurun_out/pytest_gzip.log; exit 1; }
tail -3 gpurun_out/pytest_gzip.log
