# k_walk grid / variant sweep (diagnostic): stage times of the headline bench
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -30 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
run() {
  env "$@" timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/wg.json 2> gpurun_out/wg.err || { tail -20 gpurun_out/wg.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/wg.json'));print(sys.argv[1:],d['value'],d['config']['stage_ms']['walk'],d['config']['stage_ms']['validate'],d['config']['parity'])" "$@"
}
for v in "$@"; do run $v; done
