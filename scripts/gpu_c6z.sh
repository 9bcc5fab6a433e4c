# inflate / zstd microbench + C6 stanza with every codec on the device
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/mb_inflate.py
timeout -k 10 400 python -u bench.py --workloads c6 --steps 5 --warmup 1 --no-index --no-cpu-baseline > gpurun_out/bench_c6.json 2> gpurun_out/bench_c6.err || { tail -30 gpurun_out/bench_c6.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c6.json')); c=d['config']['c6']; print(c['ms_per_step'], c['stage_ms'], c['parity'], c.get('per_codec'))"
