# Round 4 check after the reverts: GPU suite + C1 bench, then prev (8995cc2
# build) vs cur on C1/C2/C5 interleaved, and member timings prev vs cur.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_check.sh r04f "" c1
W=c1,c2,c5 bash scripts/gpu_ab.sh r04f prev cur prev cur
for V in prev cur; do
  if [ $V = cur ]; then unset RPGPU_VARIANT; else export RPGPU_VARIANT=$V; fi
  timeout -k 10 120 python scripts/mb_member_time.py gzip 3
  timeout -k 10 120 python scripts/mb_member_time.py zstd 3
done
