# Per-workload kernel trace + HBM traffic: one rocprofv3 --kernel-trace
# --stats pass of the full bench, then separate FETCH_SIZE / WRITE_SIZE
# passes per workload (c1 / c2 / c5 each in its own process, so a kernel's
# counters belong to one workload); every pass bounded, --pmc alone.
# scripts/parse_traffic.py TAG turns them into profiles/*_traffic.json.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r03}
if [ -z "${NO_TRACE:-}" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o $TAG --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-index > gpurun_out/prof_$TAG.log 2>&1
echo "trace ok"
fi
for W in ${WORKLOADS:-c1 c2 c5 c6}; do
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_${TAG}_$W -o f --output-format csv -- python3 bench.py --workloads $W --steps 2 --warmup 1 --no-cpu-baseline --no-index --stats-out gpurun_out/stats_${TAG}_$W.json > gpurun_out/pmc_fetch_${TAG}_$W.log 2>&1
echo "fetch $W ok"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_${TAG}_$W -o w --output-format csv -- python3 bench.py --workloads $W --steps 2 --warmup 1 --no-cpu-baseline --no-index > gpurun_out/pmc_write_${TAG}_$W.log 2>&1
echo "write $W ok"
done
