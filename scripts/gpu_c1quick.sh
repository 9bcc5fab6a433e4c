# discovery / planning changes: parity, then the C1 line (3 runs)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_c1q.log 2>&1 || { tail -60 gpurun_out/pytest_c1q.log; exit 1; }
tail -1 gpurun_out/pytest_c1q.log
for r in 1 2 3; do
timeout -k 10 300 python -u bench.py --workloads c1 --no-cpu-baseline --no-index > gpurun_out/bench_c1q.json 2> gpurun_out/bench_c1q.err
python -c "import json; d=json.load(open('gpurun_out/bench_c1q.json')); print(d['value'], d['config']['stage_ms'])"
done
