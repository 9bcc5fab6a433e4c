# The default bench's stanzas (c1,h2d,c2,c5,c6) under two side-stream
# setups (diagnostics): the product, and the diagnostic build with the side
# stream at default priority (RPGPU_SIDE_PRIO=0)
set -e
cd "$GRAFT_REPO_ROOT"
run() {
timeout -k 10 600 env $3 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ord_$2.json 2> gpurun_out/ord_$2.err || { tail -5 gpurun_out/ord_$2.err; exit 1; }
python3 - gpurun_out/ord_$2.json $2 <<'PY'
import json,sys
j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=j['config']
print(sys.argv[2], 'c1', j['ms_per_step'])
for k in ('c2','c5','c6'):
    if k in c: print(sys.argv[2], k, c[k]['ms_per_step'], c[k]['stage_ms'].get('resolve_plan'), c[k]['stage_ms'].get('decode'))
PY
}
run x prio "RPGPU_X=1"
run x noprio "RPGPU_VARIANT=diag RPGPU_SIDE_PRIO=0"
