#!/bin/bash
# Kernel-trace stats + PMC passes of the C2 bench (short), one counter group per run.
# Usage: tools/gpu_prof.sh <tag> [extra bench args...]
set -u
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline $*"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- $B > $OUT/kt.log 2>&1 || { echo "kt failed"; tail -5 $OUT/kt.log; exit 1; }
i=0
PMC_GROUPS=("SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE")
[ -n "${PMC_EXTRA:-}" ] && PMC_GROUPS+=("$PMC_EXTRA")
for grp in "${PMC_GROUPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- $B > $OUT/pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
find $OUT -name "*kernel_stats.csv" | head -3
exit 0
