# Instruction-cache counters of the decode kernels on a small C2 job (one bounded --pmc pass)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-sqi}
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES -d gpurun_out/${TAG}_i -o i --output-format csv -- python3 scripts/dbg_job.py c2 4 32 > gpurun_out/${TAG}_i.log 2>&1
echo "pass i ok"
