# kernel trace of the C2 diagnostic bench
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o c2 --output-format csv -- python3 scripts/bench_c2.py --workload c2 --steps 2 --warmup 1 > gpurun_out/prof_c2.log 2>&1
echo "trace ok"
