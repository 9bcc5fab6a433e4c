# final tree: PMC traffic + kernel trace (tag r04u), then the GPU suite, smoke and the exact bench command
set -e
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_traffic.sh r04u
bash scripts/gpu_final.sh r04u
