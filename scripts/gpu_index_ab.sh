# segment-index parity + A/B of the piece-parallel and serial index kernels
set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_segment_index.py tests/test_cpp_surfaces.py -x -q --timeout 120 --timeout-method thread > gpurun_out/idx.log 2>&1 || { tail -30 gpurun_out/idx.log; exit 1; }
tail -2 gpurun_out/idx.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_idx.json 2> gpurun_out/bench_idx.err
RPGPU_INDEX_SERIAL=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_idx_serial.json 2> gpurun_out/bench_idx_serial.err
python -c "
import json
for f in ('gpurun_out/bench_idx.json', 'gpurun_out/bench_idx_serial.json'):
    d = json.load(open(f)); print(f, d['value'], d['config']['segment_index'])"
