# k_walk parity (lane-walked batches of every shape) + C1 bench line
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_walk.log 2>&1 || { tail -60 gpurun_out/pytest_walk.log; exit 1; }
tail -2 gpurun_out/pytest_walk.log
timeout -k 10 300 python -u bench.py --workloads c1 --no-cpu-baseline --no-index > gpurun_out/bench_walk.json 2> gpurun_out/bench_walk.err
python -c "import json; d=json.load(open('gpurun_out/bench_walk.json')); print(d['value'], d['config']['stage_ms'])"
