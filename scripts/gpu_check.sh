# Round check: the GPU suite, smoke, the driver's exact bench command (line +
# --detail-out), then the same command under rocprofv3 --kernel-trace --stats
# (scripts/trace_summary.py reads its C1 launches).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05a}
SKIP_TESTS=${SKIP_TESTS:-}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -30 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
fi
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail-out gpurun_out/bench_detail_$TAG.json > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
wc -c gpurun_out/bench_$TAG.json
tail -c 400 gpurun_out/bench_$TAG.json
if [ -z "${NO_TRACE:-}" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o $TAG --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.log || { tail -30 gpurun_out/prof_$TAG.log; exit 1; }
echo "trace ok"
fi
if [ -n "${AB:-}" ]; then
W=c2,c5 bash scripts/gpu_ab.sh ${TAG}ab cur $AB cur $AB
fi
