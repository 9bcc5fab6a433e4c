# kernel trace of the compressed workloads only (bounded)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-c2p}
W=${2:-c2}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o $TAG --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-index --workloads $W --seg-gib 0.25 > gpurun_out/prof_$TAG.log 2>&1
echo "prof ok"
