#!/bin/bash
# C3 decode timing (tools/c3_decode_time.py) of the default library and of each error-kernel variant
# (SRC=ezrs_errors tools/build_variant.sh), twice in alternating order.
# Usage: tools/gpu_c3_ab.sh <tag> [variant names...]
set -u
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then unset EZRS_LIB_VARIANT; else export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_$v.so; fi
    timeout -k 10 120 python3 tools/c3_decode_time.py 40 >> $OUT/c3_ab.txt 2> $OUT/c3_${v}.err
    rc=$?; [ $rc -eq 0 ] || { echo "c3 $v rc=$rc"; tail -3 $OUT/c3_${v}.err; exit $rc; }
    tail -n 1 $OUT/c3_ab.txt
  done
done
unset EZRS_LIB_VARIANT
exit 0
