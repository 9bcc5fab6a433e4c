# Kernel trace of bench stanzas $W (default c6): per-kernel calls and times
# (scripts/kcalls.py) under gpurun_out/kcalls_$TAG.txt
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-tr}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o $TAG --output-format csv -- python3 bench.py --workloads ${W:-c6} --no-cpu-baseline --no-index --steps 3 --warmup 1 > gpurun_out/prof_$TAG.log 2>&1
python3 scripts/kcalls.py gpurun_out/prof_$TAG/${TAG}_kernel_trace.csv > gpurun_out/kcalls_$TAG.txt
head -30 gpurun_out/kcalls_$TAG.txt
tail -1 gpurun_out/prof_$TAG.log | cut -c1-1500
