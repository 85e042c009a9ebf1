#!/bin/bash
# r05w: BCH GPU tests on the default library (per-wave write-back of LDS corrections), then C5 timing
# A/B: default vs block-barrier write-back (bblk) vs global byte corrections (bold), 1M and 8M.
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05w; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "bch or BCH or host" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in default bprev; do
    if [ $v = default ]; then unset EZRS_LIB_VARIANT; else export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_$v.so; fi
    for n in 1048576 8388608; do
      timeout -k 10 120 python3 tools/c5_decode_time.py $n 30 >> $OUT/c5_ab.txt 2>> $OUT/c5.err || { echo "c5 $v $n failed"; tail -3 $OUT/c5.err; exit 1; }
      tail -n 1 $OUT/c5_ab.txt
    done
  done
done

exit 0
