# iteration check: GPU parity tests, headline bench, stamps breakdown; every
# GPU step bounded, chained with &&
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -30 gpurun_out/pytest_iter.log; exit 1; }
tail -2 gpurun_out/pytest_iter.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err
python3 -c "import json;d=json.load(open('gpurun_out/iter_bench.json'));print(d['value'],d['config']['stage_ms'],d['roofline']['achieved'])"
if [ -f redpanda_amd/librpgpu_stamps.so ]; then
  RPGPU_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --seg-gib 1 > gpurun_out/iter_stamps.out 2> gpurun_out/iter_stamps.err
  grep RPGPU_STAMPS gpurun_out/iter_stamps.out | tail -2 || true
fi
