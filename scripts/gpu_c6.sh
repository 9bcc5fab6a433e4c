# C6 stanza (C5 + gzip on the device + zstd on the host): gzip parity tests,
# then timing and per-codec parity counts
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "gzip or zstd" > gpurun_out/pytest_c6.log 2>&1 || { tail -40 gpurun_out/pytest_c6.log; exit 1; }
tail -1 gpurun_out/pytest_c6.log
timeout -k 10 400 python -u bench.py --workloads c6 --steps 5 --warmup 1 --no-index > gpurun_out/bench_c6.json 2> gpurun_out/bench_c6.err || { tail -30 gpurun_out/bench_c6.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c6.json')); c=d['config']['c6']; print(c['ms_per_step'], c['stage_ms'], c['parity'], c['per_codec'])"
