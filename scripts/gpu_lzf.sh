# Fast LZ4 path check: decode parity tests, then the C2/C5 stanzas with the
# fast path (librpgpu.so) against the walk/exec path (diag build, RPGPU_LZF=0)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-lzf}
K=${K:-"c2 or c5 or codec or golden or lz4 or snappy or uncompress or wire or decode"}
if [ -n "${FULL:-}" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
else
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
fi
tail -2 gpurun_out/pytest_$TAG.log
for i in 1 2; do
for V in cur old ${EXTRA:-}; do
unset RPGPU_VARIANT RPGPU_LZF
if [ "$V" = old ]; then export RPGPU_VARIANT=diag RPGPU_LZF=0; fi
if [ "$V" != old ] && [ "$V" != cur ]; then export RPGPU_VARIANT=$V; fi
timeout -k 10 300 python -u bench.py --workloads ${W:-c2,c5} --no-cpu-baseline --no-index --steps 10 --warmup 2 > gpurun_out/ab_${TAG}_${V}_$i.json 2> gpurun_out/ab_${TAG}_${V}_$i.err || { tail -30 gpurun_out/ab_${TAG}_${V}_$i.err; exit 1; }
python - gpurun_out/ab_${TAG}_${V}_$i.json $V <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = j["config"]
for k in ("c2", "c5"):
    if k in c:
        s = c[k]
        print(sys.argv[2], k, s.get("error") or (s["ms_per_step"], s["stage_ms"], s["parity"]))
PY
done
done
unset RPGPU_VARIANT RPGPU_LZF
if [ -n "${TRACE:-}" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o $TAG --output-format csv -- python3 bench.py --workloads c2,c5 --no-cpu-baseline --no-index --steps 3 --warmup 1 > gpurun_out/prof_$TAG.log 2>&1
python3 scripts/kcalls.py gpurun_out/prof_$TAG/${TAG}_kernel_trace.csv > gpurun_out/kcalls_$TAG.txt; head -14 gpurun_out/kcalls_$TAG.txt
fi
