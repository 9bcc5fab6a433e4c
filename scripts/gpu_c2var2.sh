# parity of a variant library (codec tests), then C2/C5 lines; every GPU step bounded
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -30 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
for v in "$@"; do
  if [ "$v" = "-" ]; then unset RPGPU_VARIANT; else export RPGPU_VARIANT="$v"; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "codec or decode or uncompress or host" --timeout 200 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1 || { tail -30 gpurun_out/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/pytest_$v.log)"
  for w in c2 c5; do
    timeout -k 10 300 python -u scripts/bench_c2.py --workload $w > gpurun_out/${w}_$v.json 2> gpurun_out/${w}_$v.err || { tail -20 gpurun_out/${w}_$v.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],sys.argv[3],d['stored_GBps'],d['decoded_GBps'],d['stage_ms'])" gpurun_out/${w}_$v.json $v $w
  done
done
