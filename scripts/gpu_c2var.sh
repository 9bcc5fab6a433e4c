# C2/C5 diagnostic bench per library variant ("-" = the product lib), after
# the GPU parity tests.  Every GPU step bounded, chained with &&.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -40 gpurun_out/pytest_iter.log; exit 1; }
tail -2 gpurun_out/pytest_iter.log
for v in "$@"; do
  if [ "$v" = "-" ]; then unset RPGPU_VARIANT; else export RPGPU_VARIANT="$v"; fi
  for w in c2 c5; do
    timeout -k 10 300 python -u scripts/bench_c2.py --workload $w > gpurun_out/${w}_$v.json 2> gpurun_out/${w}_$v.err || { tail -20 gpurun_out/${w}_$v.err; exit 1; }
    echo "$v $(cat gpurun_out/${w}_$v.json)"
  done
done
unset RPGPU_VARIANT
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err
python3 -c "import json;d=json.load(open('gpurun_out/iter_bench.json'));print(d['value'],d['config']['stage_ms'],d['roofline']['achieved'])"
