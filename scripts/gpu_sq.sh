# SQ instruction-mix / stall counters for k_validate (one --pmc pass each, <= 8 SQ counters)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-sq}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/${TAG}_a -o a --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --seg-gib 1 --workloads c1 --no-index > gpurun_out/${TAG}_a.log 2>&1
echo "pass a ok"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS -d gpurun_out/${TAG}_b -o b --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --seg-gib 1 --workloads c1 --no-index > gpurun_out/${TAG}_b.log 2>&1
echo "pass b ok"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/${TAG}_c -o c --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --seg-gib 1 --workloads c1 --no-index > gpurun_out/${TAG}_c.log 2>&1
echo "pass c ok"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/${TAG}_d -o d --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --seg-gib 1 --workloads c1 --no-index > gpurun_out/${TAG}_d.log 2>&1
echo "pass d ok"
