# GPU parity suite (optionally -k filter) then a C1-only bench (no CPU
# baseline); bounded steps chained with &&.  TAG names the outputs.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-chk}
K=${2:-}
if [ -n "$K" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1 || { tail -80 gpurun_out/pytest_$TAG.log; exit 1; }
else
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -80 gpurun_out/pytest_$TAG.log; exit 1; }
fi
tail -3 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -u bench.py --workloads ${3:-c1} --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python - gpurun_out/bench_$TAG.json <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = j["config"]
print("value", j["value"], "ms", j["ms_per_step"], "stages", c.get("stage_ms"), "frac_alg", c.get("hbm_fraction_whole_pipeline_alg"))
for k in ("c2", "c5", "c6"):
    if k in c:
        s = c[k]
        print(k, s.get("error") or (s["ms_per_step"], s["stage_ms"]))
PY
