# C6 stanza with its CPU baseline (8 partitions, largest-first dynamic claims)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --workloads c6 --steps 5 --warmup 1 --no-index > gpurun_out/bench_c6b.json 2> gpurun_out/bench_c6b.err || { tail -30 gpurun_out/bench_c6b.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c6b.json')); c=d['config']['c6']; print(c['ms_per_step'], c['stored_GBps'], c['decoded_GBps'], json.dumps(c['cpu_baseline']))"
