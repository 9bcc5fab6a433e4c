# A/B of library variants on the C2/C5 stanzas (parity summary included):
#   bash scripts/gpu_ab3.sh TAG VARIANT...   ("" = the product build)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
for V in prod "$@"; do
  VV=$V; [ "$V" = prod ] && VV=
  RPGPU_VARIANT=$VV timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-index --workloads c2,c5 > gpurun_out/ab3_${TAG}_$V.json 2> gpurun_out/ab3_${TAG}_$V.err || { tail -20 gpurun_out/ab3_${TAG}_$V.err; exit 1; }
  python - gpurun_out/ab3_${TAG}_$V.json "$V" <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))["config"]
for w in ("c2","c5"):
    if w in d: print(sys.argv[2], w, d[w]["ms_per_step"], "ms", {k: v for k, v in d[w]["stage_ms"].items()}, d[w]["parity"].get("all_valid"), d[w]["parity"].get("codec_ok"))
PY
done
