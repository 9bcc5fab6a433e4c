# A/B of the concurrent CRC / record walk split (diagnostic library,
# RPGPU_WALK_SPLIT = eighths of the CUs that walk), C1 only, no CPU baseline.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-split}
shift || true
for K in "$@"; do
RPGPU_VARIANT=diag RPGPU_WALK_SPLIT=$K timeout -k 10 300 python -u bench.py --workloads c1 --no-cpu-baseline --no-index --steps 20 --warmup 3 > gpurun_out/bench_${TAG}_$K.json 2> gpurun_out/bench_${TAG}_$K.err || { tail -30 gpurun_out/bench_${TAG}_$K.err; exit 1; }
python - gpurun_out/bench_${TAG}_$K.json $K <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = j["config"]
print("split", sys.argv[2], "value", j["value"], "ms", j["ms_per_step"], "stages", c.get("stage_ms"), "frac_alg", c.get("hbm_fraction_whole_pipeline_alg"), "parity", c["parity"])
PY
done
