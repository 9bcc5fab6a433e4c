# diagnostic: headline bench vs CRC-only, each GPU step bounded
set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/probe_full.json 2> gpurun_out/probe_full.err
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parse > gpurun_out/probe_crc.json 2> gpurun_out/probe_crc.err
cat gpurun_out/probe_full.json gpurun_out/probe_crc.json
