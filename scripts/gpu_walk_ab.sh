# A/B of decode-kernel variants on C2 + C5 (kernel trace per variant, bounded)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for V in "$@"; do
if [ "$V" = "base" ]; then unset RPGPU_VARIANT; else export RPGPU_VARIANT=$V; fi
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/ab_$V -o ab --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-index --workloads c2,c5 --seg-gib 0.125 > gpurun_out/ab_$V.log 2>&1
echo "== $V"; python scripts/kcalls.py gpurun_out/ab_$V/ab_kernel_trace.csv | grep -E "k_lz|k_discover|k_validate_dec|finish"
done
