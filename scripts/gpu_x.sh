# decode-engine check: debug jobs vs the oracle (also with a tiny record pool),
# GPU parity tests, then stamps of the C2/C5 decode
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-x}
timeout -k 10 150 python -u scripts/dbg_job.py c2 3 12 > gpurun_out/${TAG}_job.log 2>&1
timeout -k 10 150 python -u scripts/dbg_job.py c5 4 6 >> gpurun_out/${TAG}_job.log 2>&1
RPGPU_POOL_SLABS=40 timeout -k 10 150 python -u scripts/dbg_job.py c2 2 8 >> gpurun_out/${TAG}_job.log 2>&1
grep "bad fields" gpurun_out/${TAG}_job.log
if [ "${2:-}" != "notests" ]; then bash scripts/gpu_tests.sh $TAG; fi
W=c2,c5 bash scripts/gpu_dst_variants.sh dstamps
