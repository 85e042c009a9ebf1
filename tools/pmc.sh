#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 invocation per counter group, as the
# MI355X guide prescribes: FETCH_SIZE and WRITE_SIZE in separate passes).
# Usage: tools/pmc.sh <tag> [extra bench args]
set -u
TAG=${1:-pmc}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PMC_SETS=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
  "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
  "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC"
)
i=0
for grp in "${PMC_SETS[@]}"; do
  i=$((i+1))
  echo "== pmc pass $i: $grp"
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $OUT/p$i.log 2>&1
  rc=$?
  echo "== pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; echo "stopping"; exit $rc; fi
done
exit 0
