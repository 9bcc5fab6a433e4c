# Decode-kernel wall-clock stamps (diag builds librpgpu_<variant>.so, never the
# product): one C2 (or $W) bench stanza per variant in $VARS, the RPGPU_DSTAMPS lines
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-dst}
for V in ${VARS:-dstamps}; do
RPGPU_VARIANT=$V timeout -k 10 300 python -u bench.py --workloads ${W:-c2} --no-cpu-baseline --no-index --steps 2 --warmup 1 > gpurun_out/dst_${TAG}_$V.json 2> gpurun_out/dst_${TAG}_$V.err || { tail -30 gpurun_out/dst_${TAG}_$V.err; exit 1; }
echo "== $V"
grep -h "RPGPU_DSTAMPS" gpurun_out/dst_${TAG}_$V.err gpurun_out/dst_${TAG}_$V.json | tail -2 || true
done
