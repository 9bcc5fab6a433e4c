# LZ4 wave-walk check: decode tests on the product build and on variant
# $2 (every LZ4 block wave-walked), then the C2/C5 bench on variant $3.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-lw}
K="c2 or c5 or codec or decode or uncompress or smoke or host_path or snappy or seeded or lz4"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
RPGPU_VARIANT=$2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K" > gpurun_out/pytest_${TAG}_$2.log 2>&1 || { tail -60 gpurun_out/pytest_${TAG}_$2.log; exit 1; }
tail -1 gpurun_out/pytest_${TAG}_$2.log
for V in "" $3; do
RPGPU_VARIANT=$V timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-index --workloads c2,c5 > gpurun_out/bench_${TAG}_$V.json 2> gpurun_out/bench_${TAG}_$V.err || { tail -30 gpurun_out/bench_${TAG}_$V.err; exit 1; }
python - gpurun_out/bench_${TAG}_$V.json "$V" <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))["config"]
for w in ("c2","c5"):
    if w in d: print(sys.argv[2] or "prod", w, d[w]["ms_per_step"], "ms", {k: v for k, v in d[w]["stage_ms"].items()}, d[w]["parity"].get("all_valid"), d[w]["parity"].get("codec_ok"))
PY
done
