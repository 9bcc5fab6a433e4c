# gzip single-pass (first pass into scratch) parity + C6 timing + inflate microbench
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_surfaces.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "gzip or zstd or codec or decode or capacity or host" > gpurun_out/pytest_gz2.log 2>&1 || { tail -40 gpurun_out/pytest_gz2.log; exit 1; }
tail -1 gpurun_out/pytest_gz2.log
timeout -k 10 200 python -u scripts/mb_inflate.py
timeout -k 10 400 python -u bench.py --workloads c6 --steps 5 --warmup 1 --no-index --no-cpu-baseline > gpurun_out/bench_c6.json 2> gpurun_out/bench_c6.err || { tail -30 gpurun_out/bench_c6.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c6.json')); c=d['config']['c6']; print(c['ms_per_step'], c['stage_ms'], c['parity'])"
