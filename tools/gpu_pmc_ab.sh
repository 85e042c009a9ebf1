#!/bin/bash
# SQ counter passes of the C2 bench for the default library and a variant (EZRS_LIB_VARIANT), one
# rocprofv3 --pmc run per counter group.  Usage: tools/gpu_pmc_ab.sh <tag> [variant]
set -u
TAG=$1; V=${2:-}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
SETS=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
  "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD"
)
for lib in default $V; do
  if [ $lib = default ]; then unset EZRS_LIB_VARIANT; else export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_$lib.so; fi
  i=0
  for grp in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/$lib/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $OUT/$lib.p$i.log 2>&1
    rc=$?; echo "$lib pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/$lib.p$i.log; exit $rc; }
  done
  python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT/$lib > $OUT/$lib.summary.txt 2>&1 || true
done
exit 0
