#!/bin/bash
# Counter list + PMC passes over a short bench run (one rocprofv3 per pass).
set -u
TAG=${1:-pmc}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || { echo "list failed"; exit 1; }
grep -ioE "(SQC?_[A-Z_0-9]*(ICACHE|IFETCH|INST_LDS|LDS)[A-Z_0-9]*)" $OUT/counters.txt | sort -u > $OUT/ic.txt || true
cat $OUT/ic.txt
PMC_SETS=(
  "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
  "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_IFETCH GRBM_GUI_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for grp in "${PMC_SETS[@]}"; do
  i=$((i+1)); echo "== pass $i: $grp"
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/p$i.log 2>&1
  rc=$?; echo "== pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python tools/pmc_summary.py $OUT $OUT/summary.json > $OUT/summary.txt
exit 0
