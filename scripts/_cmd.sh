set -e
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_exp.sh "-" "sstep" "-" "sstep"
RPGPU_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --seg-gib 1 > gpurun_out/iter_stamps.out 2> gpurun_out/iter_stamps.err
grep RPGPU_STAMPS gpurun_out/iter_stamps.out | tail -1
