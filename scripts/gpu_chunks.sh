# discovery chunk-size sweep of the headline bench (diagnostic)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for c in "$@"; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --chunk-kib $c > gpurun_out/chunk_$c.json 2> gpurun_out/chunk_$c.err || { tail -20 gpurun_out/chunk_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/chunk_$c.json'));print($c,d['value'],d['config']['stage_ms'])"
done
