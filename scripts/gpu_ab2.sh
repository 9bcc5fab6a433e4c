# decode A/B (kernel trace per variant) + decode stamps of C2 alone
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_walk_ab.sh "$@"
export RPGPU_VARIANT=dstamps
timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-index --workloads c2 > gpurun_out/dst_c2.out 2> gpurun_out/dst_c2.err
echo "== dstamps c2"; grep RPGPU_DSTAMPS gpurun_out/dst_c2.out | tail -3
