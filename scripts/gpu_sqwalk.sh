# SQ / TA / TCP counters for k_walk (one --pmc pass each)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-sqw}
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --seg-gib 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/${TAG}_a -o a --output-format csv -- $B > gpurun_out/${TAG}_a.log 2>&1
echo "pass a ok"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS -d gpurun_out/${TAG}_b -o b --output-format csv -- $B > gpurun_out/${TAG}_b.log 2>&1
echo "pass b ok"
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE -d gpurun_out/${TAG}_c -o c --output-format csv -- $B > gpurun_out/${TAG}_c.log 2>&1
echo "pass c ok"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d gpurun_out/${TAG}_d -o d --output-format csv -- $B > gpurun_out/${TAG}_d.log 2>&1
echo "pass d ok"
