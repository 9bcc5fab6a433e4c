# Round-6 experiment call: targeted LZ4/snappy parity tests on the product
# build, then an A/B of bench stanzas (scripts/gpu_ab.sh) over $AB variants
# and decode stamps (scripts/gpu_dstamps.sh) over $DVARS (diagnostic builds).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r06x}
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_lz4_walk.py tests/test_gpu_parity.py} -m gpu -x -v --timeout 240 --timeout-method thread -k "${TESTK:-lz4 or c2_recipe or c5_recipe or codec_mix or raw_snappy or uncompress or golden}" > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
fi
if [ -n "${AB:-}" ]; then
bash scripts/gpu_ab.sh ${TAG}ab $AB
fi
if [ -n "${DVARS:-}" ]; then
VARS="$DVARS" bash scripts/gpu_dstamps.sh ${TAG}
fi
