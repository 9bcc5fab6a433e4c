# parity tests, then the headline bench with and without a diagnostic switch
# (A/B).  Usage: gpu_ab.sh VAR=VALUE ...  Every GPU step bounded, chained.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -30 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_base.json 2> gpurun_out/ab_base.err || { tail -20 gpurun_out/ab_base.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/ab_base.json'));print('base',d['value'],d['config']['stage_ms'],d['config']['parity'])"
for kv in "$@"; do
  env "$kv" timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_var.json 2> gpurun_out/ab_var.err || { tail -20 gpurun_out/ab_var.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_var.json'));print('$kv',d['value'],d['config']['stage_ms'],d['config']['parity'])"
done
