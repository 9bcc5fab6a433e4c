# bench + kernel-trace profile; each GPU step bounded, chained with &&
set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_r01.json 2> gpurun_out/bench_r01.err
echo "bench ok"
cat gpurun_out/bench_r01.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01 -o r01 --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_r01.log 2>&1
echo "prof ok"
find gpurun_out/prof_r01 -name "*stats*" | head
