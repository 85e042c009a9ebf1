#!/bin/bash
# r05j: full GPU suite on the default library (BM log cache, early DMA off), C3 decode A/B of the
# error-kernel variants (no cache; timing ablations stopping after each phase), tile-kernel stamps.
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05j; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
tools/gpu_c3_ab.sh r05j enocache es4 es1 es2 es3 || exit 1
for b in pq_stamps pq_stamps_early pq_stamps_nodma; do
  timeout -k 10 60 tools/micro/$b > $OUT/$b.txt 2>&1 || { echo "$b failed"; exit 1; }
done
grep -h -E "decode|tile [0-3]" $OUT/pq_stamps*.txt
exit 0
