set -e
cd "$GRAFT_REPO_ROOT"
for p in 1 2 4 16; do
timeout -k 10 120 python -u bench.py --workloads c1 --no-cpu-baseline --no-index --seg-gib 0.0625 --partitions $p --steps 20 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print($p, c['records_per_gpu'], c['stage_ms'])"
done
