# decode parity (C2/C5 recipes, codec mixes) then the C2 / C5 stanzas
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "c2 or c5 or codec or decode or snappy or lz4 or linked" > gpurun_out/pytest_dec.log 2>&1 || { tail -40 gpurun_out/pytest_dec.log; exit 1; }
tail -1 gpurun_out/pytest_dec.log
timeout -k 10 400 python -u bench.py --workloads c2,c5 --steps 5 --warmup 1 --no-cpu-baseline --no-index > gpurun_out/bench_dec.json 2> gpurun_out/bench_dec.err
python -c "import json; d=json.load(open('gpurun_out/bench_dec.json'))['config']; [print(k, d[k]['ms_per_step'], d[k]['stage_ms']) for k in ('c2','c5')]"
