# A/B of bench stanzas $W (default c2,c5) over variants: each argument after
# the tag is NAME=VARIANT[:ENV=VAL[,ENV=VAL]] (VARIANT "cur" = librpgpu.so),
# two rounds, per-stanza ms_per_step / stage_ms / parity lines (diagnostics)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1
shift
for i in 1 2; do
for spec in "$@"; do
name=${spec%%=*}
rest=${spec#*=}
var=${rest%%:*}
envs=""
[ "$rest" != "$var" ] && envs=${rest#*:}
(
unset RPGPU_VARIANT
[ "$var" != cur ] && export RPGPU_VARIANT=$var
for kv in ${envs//,/ }; do export "$kv"; done
timeout -k 10 300 python -u bench.py --workloads ${W:-c2,c5} --no-cpu-baseline --no-index --steps 10 --warmup 2 > gpurun_out/ab_${TAG}_${name}_$i.json 2> gpurun_out/ab_${TAG}_${name}_$i.err
) || { tail -30 gpurun_out/ab_${TAG}_${name}_$i.err; exit 1; }
python - gpurun_out/ab_${TAG}_${name}_$i.json $name <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = j["config"]
for k in ("c1", "c2", "c5", "c6"):
    if k in c:
        s = c[k]
        print(sys.argv[2], k, s.get("error") or (s["ms_per_step"], s["stage_ms"].get("decode"), s["stage_ms"].get("resolve_plan"), s["parity"].get("all_valid", s["parity"])))
PY
done
done
