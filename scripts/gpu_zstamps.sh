# zstd decoder phase stamps (RPGPU_ZSTAMPS diagnostic build) on the zstd microbench shapes, then parity + C6
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
RPGPU_VARIANT=zst timeout -k 10 300 python -u scripts/mb_inflate.py > gpurun_out/zstamps.out 2>&1 || { tail -30 gpurun_out/zstamps.out; exit 1; }
grep -E "RPGPU_ZSTAMPS payloads=[1-9]|^zstd" gpurun_out/zstamps.out | head -20
bash scripts/gpu_zstd2.sh
