# Round end on the final tree: PMC traffic + kernel trace of the bench
# (scripts/gpu_traffic.sh TAG; then scripts/parse_traffic.py TAG here), the
# GPU suite, smoke() and the driver's exact bench command (scripts/gpu_final.sh).
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r04}
bash scripts/gpu_traffic.sh $TAG
bash scripts/gpu_final.sh $TAG
