# SQ counters of the LZ4 decode kernels (k_lz_walk, k_lz_exec, k_validate_decoded)
# on the C2 bench stanza (8 x 1.5 GiB): one --pmc pass each, bounded (diagnostics)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-sql}
J="python3 bench.py --workloads c2 --steps 1 --warmup 0 --no-cpu-baseline --no-index"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_k -o k --output-format csv -- $J > gpurun_out/${TAG}_k.log 2>&1
echo "pass k ok"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/${TAG}_a -o a --output-format csv -- $J > gpurun_out/${TAG}_a.log 2>&1
echo "pass a ok"
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS -d gpurun_out/${TAG}_b -o b --output-format csv -- $J > gpurun_out/${TAG}_b.log 2>&1
echo "pass b ok"
timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU -d gpurun_out/${TAG}_c -o c --output-format csv -- $J > gpurun_out/${TAG}_c.log 2>&1
echo "pass c ok"
for k in ${KS:-k_lz_walk k_lz_exec k_validate_decoded}; do echo "== $k"; python3 scripts/sq_summary.py $TAG $k; done
