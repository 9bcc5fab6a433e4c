set -e
cd "$GRAFT_REPO_ROOT"
RPGPU_CHECKED=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --seg-gib 0.5 --no-cpu-baseline > gpurun_out/chk2.out 2> gpurun_out/chk2.err
echo "checked: $(grep -c RPGPU_CHECK gpurun_out/chk2.out || true) violations"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest gpu ok"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_r01.json 2> gpurun_out/bench_r01.err
echo "bench ok"
cat gpurun_out/bench_r01.json
