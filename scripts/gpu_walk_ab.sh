# k_walk A/B: variants of the walk's cache policy knobs (diagnostic builds), C1
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in "" ntidx aux0 aux1; do
RPGPU_VARIANT=$v timeout -k 10 200 python -u bench.py --workloads c1 --no-cpu-baseline --no-index --steps 10 > gpurun_out/bench_wab.json 2> gpurun_out/bench_wab.err
python -c "import json; d=json.load(open('gpurun_out/bench_wab.json')); print('variant [$v]', d['value'], d['config']['stage_ms'])"
done
