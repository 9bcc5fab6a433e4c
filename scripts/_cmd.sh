set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -40 gpurun_out/pytest_iter.log; exit 1; }
tail -2 gpurun_out/pytest_iter.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u scripts/bench_c2.py --workload c2 > gpurun_out/c2.json 2> gpurun_out/c2.err || { tail -20 gpurun_out/c2.err; exit 1; }
cat gpurun_out/c2.json
timeout -k 10 300 python -u scripts/bench_c2.py --workload c5 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -20 gpurun_out/c5.err; exit 1; }
cat gpurun_out/c5.json
bash scripts/gpu_exp.sh "-"
