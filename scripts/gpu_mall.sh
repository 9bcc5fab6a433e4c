set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for cfg in "0.0625 2" "0.25 2" "1 4"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --seg-gib $1 --partitions $2 > gpurun_out/mall.json 2> gpurun_out/mall.err || { tail -20 gpurun_out/mall.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/mall.json'));c=d['config'];print('$cfg',d['value'],c['batches_per_gpu'],c['stage_ms'])"
done
