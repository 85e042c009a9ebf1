#!/bin/bash
# C5 traffic passes (FETCH_SIZE / WRITE_SIZE, one run each) at 1 M and 8 M codewords.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06j; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-extras --workload c5"
for n in 1048576 8388608; do
  for grp in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_c5_$n/$grp -o run -- $B --ncw $n --steps 2 --warmup 1 \
        > $OUT/pmc_c5_${n}_$grp.log 2>&1 || { echo "pass $n $grp failed"; tail -3 $OUT/pmc_c5_${n}_$grp.log; exit 1; }
    echo "pass $n $grp ok"
  done
done
exit 0
