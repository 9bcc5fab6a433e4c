# diagnostic: k_walk time vs batch size (16 KiB stride vs non-power-of-two strides)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for bb in 16384 16448 16000 15000; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --batch-bytes $bb > gpurun_out/camp.json 2> gpurun_out/camp.err || { tail -20 gpurun_out/camp.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/camp.json'));c=d['config'];print($bb,d['value'],c['batches_per_gpu'],c['records_per_gpu'],c['stage_ms'],c['parity'])"
done
