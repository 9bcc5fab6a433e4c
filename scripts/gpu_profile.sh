# rocprofv3 kernel trace + PMC passes of the headline bench; each pass is its
# own bounded run (--pmc alone, no trace domains beside it)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o $TAG --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
echo "trace ok"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o fetch --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch_$TAG.log 2>&1
echo "fetch ok"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o write --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write_$TAG.log 2>&1
echo "write ok"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetchnp_$TAG -o fetchnp --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parse > gpurun_out/pmc_fetchnp_$TAG.log 2>&1
echo "fetch crc-only ok"
