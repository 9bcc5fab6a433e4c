# mb_snappy timings, kernel trace and two SQ counter passes (bounded, chained)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-mb}
timeout -k 10 120 python -u scripts/mb_snappy.py 5
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_k -o k --output-format csv -- python3 scripts/mb_snappy.py 2 > gpurun_out/${TAG}_k.log 2>&1
python scripts/kcalls.py gpurun_out/${TAG}_k/k_kernel_trace.csv | head -6
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/${TAG}_a -o a --output-format csv -- python3 scripts/mb_snappy.py 2 > gpurun_out/${TAG}_a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS -d gpurun_out/${TAG}_b -o b --output-format csv -- python3 scripts/mb_snappy.py 2 > gpurun_out/${TAG}_b.log 2>&1
echo "## k_lz_walk"; python scripts/sq_summary.py $TAG k_lz_walk
echo "## k_lz_exec"; python scripts/sq_summary.py $TAG k_lz_exec
