set -e
cd "$GRAFT_REPO_ROOT"
RPGPU_STAMPS=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --seg-gib 1 > gpurun_out/stamps.out 2> gpurun_out/stamps.err
grep RPGPU_STAMPS gpurun_out/stamps.out | tail -2
RPGPU_STAMPS=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --seg-gib 1 --no-parse > gpurun_out/stamps2.out 2> gpurun_out/stamps2.err
grep RPGPU_STAMPS gpurun_out/stamps2.out | tail -2
