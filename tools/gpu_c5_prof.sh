#!/bin/bash
# C5 kernel traces and FETCH_SIZE / WRITE_SIZE passes (one counter group per run) at 1 M and 8 M.
# Usage: tools/gpu_c5_prof.sh <tag>
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-extras --workload c5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- $B --steps 20 --warmup 3 > $OUT/prof_c5.log 2>&1 || { echo "trace 1M failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5_8m -o run -- $B --ncw 8388608 --steps 5 --warmup 1 > $OUT/prof_c5_8m.log 2>&1 || { echo "trace 8M failed"; exit 1; }
for n in 1048576 8388608; do
  d=$OUT/pmc_c5; [ $n = 8388608 ] && d=$OUT/pmc_c5_8m
  for grp in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $d/$grp -o run -- $B --ncw $n --steps 2 --warmup 1 \
        > $d.$grp.log 2>&1 || { echo "pass $n $grp failed"; tail -3 $d.$grp.log; exit 1; }
  done
done
echo done
exit 0
