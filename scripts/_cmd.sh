set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -30 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
bash scripts/gpu_exp.sh "-" "base" "-" "base"
RPGPU_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --seg-gib 1 > gpurun_out/iter_stamps.out 2> gpurun_out/iter_stamps.err
grep RPGPU_STAMPS gpurun_out/iter_stamps.out | tail -1
