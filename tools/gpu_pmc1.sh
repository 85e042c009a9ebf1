#!/bin/bash
# One rocprofv3 PMC pass (counters in $2) over a short bench run; summary to stdout.
# Usage: tools/gpu_pmc1.sh <tag> "<counters>" [bench args...]
set -u
TAG=$1; CNT=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline $*"
timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d $OUT/pmc -o run -- $B > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT
