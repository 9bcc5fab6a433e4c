# kernel-trace profile of the headline bench including the segment-index pass;
# each GPU step bounded, chained with &&
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01l -o r01l --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_r01l.log 2>&1
echo "prof ok"
find gpurun_out/prof_r01l -name "*stats*"
