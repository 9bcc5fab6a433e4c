# zstd parse/execute split: GPU suite, member timing, C6 stanza; then the
# 8 KiB exec ring A/B on C2 / C5.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r04h.log 2>&1 || { tail -60 gpurun_out/pytest_r04h.log; exit 1; }
tail -2 gpurun_out/pytest_r04h.log
timeout -k 10 120 python scripts/mb_member_time.py zstd 3
timeout -k 10 120 python scripts/mb_member_time.py gzip 3
timeout -k 10 300 python -u bench.py --workloads c6 --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/bench_c6_r04h.json 2> gpurun_out/bench_c6_r04h.err || { tail -30 gpurun_out/bench_c6_r04h.err; exit 1; }
python - gpurun_out/bench_c6_r04h.json <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = j["config"]["c6"]
print("c6", s.get("error") or (s["ms_per_step"], s["stage_ms"], s.get("parity"), s.get("member_pass")))
PY
RPGPU_VARIANT=ring8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_ring8.log 2>&1 || { tail -40 gpurun_out/pytest_ring8.log; exit 1; }
tail -2 gpurun_out/pytest_ring8.log
W=c2,c5 bash scripts/gpu_ab.sh r04h cur ring8 cur ring8
