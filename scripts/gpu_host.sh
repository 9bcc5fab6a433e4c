# host path: parity test + PCIe-inclusive rate (pinned and pageable)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "host_path" --timeout 200 --timeout-method thread > gpurun_out/pytest_host.log 2>&1 || { tail -40 gpurun_out/pytest_host.log; exit 1; }
tail -1 gpurun_out/pytest_host.log
timeout -k 10 300 python -u scripts/bench_host.py > gpurun_out/bench_host.json 2> gpurun_out/bench_host.err || { tail -20 gpurun_out/bench_host.err; exit 1; }
cat gpurun_out/bench_host.json
timeout -k 10 300 python -u scripts/bench_host.py --pageable > gpurun_out/bench_host_pg.json 2> gpurun_out/bench_host_pg.err || { tail -20 gpurun_out/bench_host_pg.err; exit 1; }
cat gpurun_out/bench_host_pg.json
