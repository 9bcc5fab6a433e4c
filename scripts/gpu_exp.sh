# run the headline bench for several library variants / flags; prints one
# summary line per run.  Args: "variant|flags" items ("-" = the product lib).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
i=0
for item in "$@"; do
  v="${item%%|*}"; f="${item#*|}"; [ "$f" = "$item" ] && f=""
  if [ "$v" = "-" ]; then unset RPGPU_VARIANT; else export RPGPU_VARIANT="$v"; fi
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline $f > gpurun_out/exp_$i.json 2> gpurun_out/exp_$i.err
  python3 -c "import json,sys;d=json.load(open('gpurun_out/exp_$i.json'));print('$v','$f',d['value'],'validate_ms',d['config']['stage_ms']['validate'],'ok',d['config']['parity'])"
  i=$((i+1))
done
