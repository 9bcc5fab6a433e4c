# decode check: the decode-path GPU parity tests, then the C2/C5 bench
# stanzas (no CPU baseline) and a kernel trace of them.  Bounded, chained.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-dec}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "c2 or c5 or codec or decode or uncompress or smoke or host_path or snappy or seeded" > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-index --workloads c2,c5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python - gpurun_out/bench_$TAG.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))["config"]
for w in ("c2","c5"):
    if w in d: print(w, d[w]["ms_per_step"], "ms", d[w]["decoded_GBps"], "GB/s dec", {k: v for k, v in d[w]["stage_ms"].items()}, d[w]["parity"])
PY
if [ "${2:-}" = "prof" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o $TAG --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-index --workloads c2,c5 > gpurun_out/prof_$TAG.log 2>&1
python scripts/kcalls.py gpurun_out/prof_$TAG/${TAG}_kernel_trace.csv
fi
