# decode-kernel stamps (RPGPU_DSTAMPS builds) for experiment variants on C2
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for V in "$@"; do
RPGPU_VARIANT=$V timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-index --workloads ${W:-c2} > gpurun_out/dstv_$V.out 2> gpurun_out/dstv_$V.err
echo "== $V"; grep RPGPU_DSTAMPS gpurun_out/dstv_$V.out | tail -3
done
