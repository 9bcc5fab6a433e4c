# host-path measurements: rpgpu_validate_host (Python engine) and the C++
# log_replayer::recover surface over 1 GiB host segments; bounded steps
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03}
timeout -k 10 300 python -u scripts/bench_host.py --partitions 8 --seg-gib 1 --reps 3 > gpurun_out/host_$TAG.json 2> gpurun_out/host_$TAG.err
cat gpurun_out/host_$TAG.json
timeout -k 10 300 python -u scripts/bench_host.py --partitions 8 --seg-gib 1 --reps 3 --no-records > gpurun_out/host_norec_$TAG.json 2>> gpurun_out/host_$TAG.err
cat gpurun_out/host_norec_$TAG.json
timeout -k 10 300 python -u scripts/bench_replayer.py 2 3 > gpurun_out/replayer_$TAG.json 2>> gpurun_out/host_$TAG.err
cat gpurun_out/replayer_$TAG.json
