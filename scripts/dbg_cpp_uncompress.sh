# Debug: the C++ compressor::uncompress surface per codec fixture, bounded
cd "$GRAFT_REPO_ROOT"
LOG=gpurun_out/dbg_cpp.log
for f in tests/golden/codecs/*.bin; do
  n=$(basename $f .bin)
  c=3; case $n in snappy*) c=2;; esac
  echo -n "$n ... " >> $LOG
  timeout -k 5 30 tests/cpp/_bin/surfaces_test uncompress $c $f /tmp/o.bin >> $LOG 2>&1
  rc=$?
  echo " rc=$rc" >> $LOG
  if [ $rc -ge 124 ]; then exit 1; fi
done
