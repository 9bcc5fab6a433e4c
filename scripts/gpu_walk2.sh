# decode tests on the product build and on variant lw0 (every LZ4 block
# wave-walked), the C2/C5 bench, then the C5 decode stamps
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-w2}
K="c2 or c5 or codec or decode or uncompress or smoke or host_path or snappy or seeded or lz4"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
RPGPU_VARIANT=lw0 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > gpurun_out/pytest_${TAG}_lw0.log 2>&1 || { tail -40 gpurun_out/pytest_${TAG}_lw0.log; exit 1; }
tail -1 gpurun_out/pytest_${TAG}_lw0.log
bash scripts/gpu_ab3.sh $TAG
W=c5 bash scripts/gpu_dst_variants.sh dstamps
