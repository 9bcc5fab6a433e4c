# Rehearsal of bench.py's N > 1 path on ONE card: two torchrun ranks share
# cuda:0, the gather goes through gloo (host-staged), and --check-gather has
# rank 0 compare the gathered job with one job over every partition.  Then
# the exact driver command at N = 1.  Every GPU step bounded, chained.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r04}
for G in records index bitmap; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 --seg-gib 0.25 --dist-backend gloo \
  --gather $G --check-gather --no-cpu-baseline > gpurun_out/bench_n2_${G}_$TAG.json 2> gpurun_out/bench_n2_${G}_$TAG.err \
  || { tail -40 gpurun_out/bench_n2_${G}_$TAG.err; exit 1; }
python - gpurun_out/bench_n2_${G}_$TAG.json <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = j["config"]
print(sys.argv[1], "value", j["value"], "gather_check", c["gather_check"], "gathered", c["gathered_records"])
PY
done
if [ "${2:-}" = "n1" ]; then
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
fi
