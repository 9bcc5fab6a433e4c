# FETCH_SIZE calibration for k_validate (MI355X_MICROARCH.md §HBM: only wide
# coalesced streams are calibrated).  CRC-only run (window loads only, dwordx4
# per lane) vs the full run (adds the record walk's scalar / 32 B loads).
# Each pass is its own bounded run, --pmc only.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetchnp_$TAG -o fetchnp --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parse > gpurun_out/pmc_fetchnp_$TAG.log 2>&1
echo "fetch no-parse ok"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o fetch --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch_$TAG.log 2>&1
echo "fetch ok"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o write --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write_$TAG.log 2>&1
echo "write ok"
