# discovery check: the parity tests that exercise the chain discovery, then
# the C1 + C2 stanzas (no CPU baseline).  Bounded, chained.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-disc}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_surfaces.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-index --workloads ${W:-c1,c2} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python - gpurun_out/bench_$TAG.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
print("c1", d["value"], d["ms_per_step"], d["config"]["stage_ms"])
for w in ("c2","c5"):
    if w in d["config"]: c=d["config"][w]; print(w, c["ms_per_step"], c["decoded_GBps"], c["stage_ms"])
PY
