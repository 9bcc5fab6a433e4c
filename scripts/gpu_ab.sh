# A/B of library variants on one box: C1 bench per variant, interleaved
# (cur = librpgpu.so, NAME = librpgpu_NAME.so).  Diagnostics only.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
W=${W:-c1}
i=0
for V in "$@"; do
i=$((i+1))
if [ "$V" = cur ]; then unset RPGPU_VARIANT; else export RPGPU_VARIANT=$V; fi
timeout -k 10 300 python -u bench.py --workloads $W --no-cpu-baseline --no-index --steps 20 --warmup 3 > gpurun_out/ab_${TAG}_$i.json 2> gpurun_out/ab_${TAG}_$i.err || { tail -30 gpurun_out/ab_${TAG}_$i.err; exit 1; }
python - gpurun_out/ab_${TAG}_$i.json $V <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = j["config"]
if j["value"]:
    print(sys.argv[2], "value", j["value"], "ms", j["ms_per_step"], "stages", c.get("stage_ms"), "parity", c["parity"])
for k in ("c2", "c5", "c6"):
    if k in c:
        s = c[k]
        print(sys.argv[2], k, s.get("error") or (s["ms_per_step"], s["stage_ms"]))
PY
done
unset RPGPU_VARIANT
