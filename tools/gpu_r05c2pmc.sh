#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of the C2 command (one counter per run) -> gpurun_out/$TAG/pmc_c2
set -u
TAG=${1:-r05f}; OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 timeout -s KILL 170 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_c2/$grp -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-extras --steps 5 --warmup 2 > $OUT/pmc_c2_$grp.log 2>&1
  rc=$?; echo "pmc_c2_$grp rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/pmc_c2_$grp.log; exit $rc; }
done
exit 0
