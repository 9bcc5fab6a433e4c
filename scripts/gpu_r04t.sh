set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r04t.log 2>&1 || { tail -60 gpurun_out/pytest_r04t.log; exit 1; }
tail -2 gpurun_out/pytest_r04t.log
timeout -k 10 120 python scripts/mb_member_time.py zstd 3
timeout -k 10 300 python -u bench.py --workloads c6 --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/bench_c6_r04t.json 2> gpurun_out/bench_c6_r04t.err || { tail -30 gpurun_out/bench_c6_r04t.err; exit 1; }
python - gpurun_out/bench_c6_r04t.json <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = j["config"]["c6"]
print("c6", s.get("error") or (s["ms_per_step"], s["stage_ms"], s.get("parity"), s.get("member_pass")))
PY
