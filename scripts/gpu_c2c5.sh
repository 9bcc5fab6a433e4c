# codec parity tests, then C2 / C5 diagnostic bench lines (product lib), each bounded
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -30 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
for w in c2 c5; do
  timeout -k 10 300 python -u scripts/bench_c2.py --workload $w > gpurun_out/${w}.json 2> gpurun_out/${w}.err || { tail -20 gpurun_out/${w}.err; exit 1; }
  cat gpurun_out/${w}.json
done
