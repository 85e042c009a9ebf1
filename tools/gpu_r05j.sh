#!/bin/bash
# r05j: full GPU suite on the default library (BM log cache, early DMA off, BCH corrections in LDS,
# compacted host rows), the error-path parity tests on the coalesced-correction variant, C3 decode
# A/B of the error-kernel variants (timing ablations stopping after each phase), tile-kernel stamps.
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05j; mkdir -p $OUT
export TMPDIR=/tmp
if [ "${SKIP_SUITE:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_eco8.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q \
    --timeout 200 --timeout-method thread -k "(c3 or erasure or bulk or karn or full_length or shard or positions) and not abi" > $OUT/pytest_eco8.log 2>&1
rc=$?; echo "pytest eco8 rc=$rc"; tail -n 3 $OUT/pytest_eco8.log; [ $rc -eq 0 ] || exit $rc
tools/gpu_c3_ab.sh r05j enocache ech8 eco eco8 es4 es1 es2 es3 || exit 1
for b in pq_stamps pq_stamps_early pq_stamps_nodma; do
  timeout -k 10 60 tools/micro/$b > $OUT/$b.txt 2>&1 || { echo "$b failed"; exit 1; }
done
grep -h -E "decode|tile [0-3]" $OUT/pq_stamps*.txt
exit 0
