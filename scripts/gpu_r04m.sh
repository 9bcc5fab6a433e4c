set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for V in cur gzno cur gzno; do
  if [ $V = cur ]; then unset RPGPU_VARIANT; else export RPGPU_VARIANT=$V; fi
  timeout -k 10 120 python scripts/mb_member_time.py gzip 3
done
unset RPGPU_VARIANT
timeout -k 10 120 python scripts/mb_member_time.py zstd 3
