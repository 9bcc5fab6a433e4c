# decode-engine cycle stamps (RPGPU_DSTAMPS build, diagnostics only) on C2 and C5
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
RPGPU_VARIANT=dstamps timeout -k 10 300 python -u bench.py --workloads c2 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/dstamps_c2.out 2> gpurun_out/dstamps_c2.err
grep RPGPU_DSTAMPS gpurun_out/dstamps_c2.out | tail -4
RPGPU_VARIANT=dstamps timeout -k 10 300 python -u bench.py --workloads c5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/dstamps_c5.out 2> gpurun_out/dstamps_c5.err
grep RPGPU_DSTAMPS gpurun_out/dstamps_c5.out | tail -4
