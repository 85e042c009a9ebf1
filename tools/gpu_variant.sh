#!/bin/bash
# A/B of the RS(255,223) syndrome kernel variants (EZRS_PS_VARIANT): bench + kernel trace + FETCH.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-variant}; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for v in pair group4; do
  EZRS_PS_VARIANT=$v timeout -k 10 200 python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v failed"; tail -3 $OUT/bench_$v.err; exit 1; }
  cut -c1-200 $OUT/bench_$v.json; grep -o '"avg_ms": {[^}]*}' $OUT/bench_$v.json
done
export EZRS_PS_VARIANT=group4
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_g4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/kt_g4.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_g4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_g4.log 2>&1 || exit 1
exit 0
