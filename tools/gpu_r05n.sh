#!/bin/bash
# r05n: FETCH_SIZE / WRITE_SIZE of the C5 kernels (1M codewords) for the default library and the
# global-byte-correction variant (bold), one counter per rocprofv3 run; then the same for C3.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05n; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for v in default bold; do
  if [ $v = default ]; then unset EZRS_LIB_VARIANT; else export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_$v.so; fi
  for grp in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/c5_$v/p_$grp -o run -- python3 $GRAFT_REPO_ROOT/tools/c5_decode_time.py 1048576 3 > $OUT/c5_${v}_$grp.log 2>&1 || { echo "pmc $v $grp failed"; tail -3 $OUT/c5_${v}_$grp.log; exit 1; }
  done
  python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT/c5_$v > $OUT/c5_${v}_summary.txt 2>&1
  grep -A4 "bch" $OUT/c5_${v}_summary.txt | head -20
done
exit 0
