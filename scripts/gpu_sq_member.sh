# SQ counters of the member pass (k_members_first) on 1 MiB gzip / zstd members
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for C in zstd gzip; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/sqm_${C}_a -o a --output-format csv -- python3 scripts/mb_member.py $C > gpurun_out/sqm_${C}_a.log 2>&1
echo "$C pass a ok"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS -d gpurun_out/sqm_${C}_b -o b --output-format csv -- python3 scripts/mb_member.py $C > gpurun_out/sqm_${C}_b.log 2>&1
echo "$C pass b ok"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/sqm_${C}_c -o c --output-format csv -- python3 scripts/mb_member.py $C > gpurun_out/sqm_${C}_c.log 2>&1
echo "$C pass c ok"
done
timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES -d gpurun_out/sqm_ic -o ic --output-format csv -- python3 scripts/mb_member.py zstd > gpurun_out/sqm_ic.log 2>&1 || echo "icache pass failed"
echo "ic done"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/sqm_kt -o kt --output-format csv -- python3 scripts/mb_member.py zstd 2 > gpurun_out/sqm_kt.log 2>&1
echo "kt ok"
