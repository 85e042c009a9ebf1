#!/bin/bash
# r05c4: C4 decode timing (tools/c4_decode_time.py, device-generated 8 errors + 4 erasures) of the
# error kernel's waves per workgroup: 16 (default, spills), 12, 8; twice in alternating order.
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05c4; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in default ew12 ew8; do
    if [ $v = default ]; then unset EZRS_LIB_VARIANT; else export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_$v.so; fi
    echo -n "$rep $v: " >> $OUT/c4_ab.txt
    timeout -k 10 150 python3 tools/c4_decode_time.py 65536 5 >> $OUT/c4_ab.txt 2>> $OUT/c4.err || { echo "c4 $v failed"; tail -5 $OUT/c4.err; exit 1; }
    tail -n 1 $OUT/c4_ab.txt
  done
done
exit 0
