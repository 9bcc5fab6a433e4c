# round check + kernel-trace profile; every GPU step bounded, chained with &&
set -e
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_round.sh
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01r -o r01r --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_r01r.log 2>&1
echo "prof ok"
