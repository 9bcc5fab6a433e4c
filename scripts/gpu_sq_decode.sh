# SQ counters of the decode kernels on a small C2 job (one --pmc pass each, bounded)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-sqd}
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/${TAG}_a -o a --output-format csv -- python3 scripts/dbg_job.py c2 4 32 > gpurun_out/${TAG}_a.log 2>&1
echo "pass a ok"
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS -d gpurun_out/${TAG}_b -o b --output-format csv -- python3 scripts/dbg_job.py c2 4 32 > gpurun_out/${TAG}_b.log 2>&1
echo "pass b ok"
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INSTS_FLAT SQ_INSTS_FLAT_LDS_ONLY GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/${TAG}_c -o c --output-format csv -- python3 scripts/dbg_job.py c2 4 32 > gpurun_out/${TAG}_c.log 2>&1
echo "pass c ok"
if [ "${2:-}" = "tcp" ]; then
timeout -s KILL 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum -d gpurun_out/${TAG}_d -o d --output-format csv -- python3 scripts/dbg_job.py c2 4 32 > gpurun_out/${TAG}_d.log 2>&1
echo "pass d ok"
fi
