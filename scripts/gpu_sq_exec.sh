# SQ / LDS counters of k_lz_exec and k_lz_walk on a small C2 job (one --pmc pass each, bounded)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-sqx}
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_k -o k --output-format csv -- python3 scripts/dbg_job.py c2 4 32 > gpurun_out/${TAG}_k.log 2>&1
echo "pass k ok"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/${TAG}_a -o a --output-format csv -- python3 scripts/dbg_job.py c2 4 32 > gpurun_out/${TAG}_a.log 2>&1
echo "pass a ok"
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS -d gpurun_out/${TAG}_b -o b --output-format csv -- python3 scripts/dbg_job.py c2 4 32 > gpurun_out/${TAG}_b.log 2>&1
echo "pass b ok"
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT -d gpurun_out/${TAG}_c -o c --output-format csv -- python3 scripts/dbg_job.py c2 4 32 > gpurun_out/${TAG}_c.log 2>&1
echo "pass c ok"
