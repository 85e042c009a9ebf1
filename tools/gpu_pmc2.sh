#!/bin/bash
# SQ/LDS/TA counter passes over a short C2 bench (one rocprofv3 run per counter group, at most 8 SQ
# counters each), then the phase stamps of the tile kernel on random data (tools/micro/pq_stamps).
# Usage: tools/gpu_pmc2.sh <tag> [extra bench args]
set -u
TAG=${1:-pmc2}; shift || true
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras $*"
GROUPS_=(
  "SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_MISC"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_UNALIGNED_STALL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_ACTIVE_INST_VMEM"
  "SQ_INST_CYCLES_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_VALU"
)
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $B > $OUT/p$i.log 2>&1 || { echo "pmc $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
if [ -x tools/micro/pq_stamps ]; then
  timeout -k 10 60 tools/micro/pq_stamps > $OUT/pq_stamps_dec.txt 2>&1 || { echo "stamps failed"; exit 1; }
  timeout -k 10 60 tools/micro/pq_stamps 1 > $OUT/pq_stamps_enc.txt 2>&1 || { echo "stamps enc failed"; exit 1; }
  cat $OUT/pq_stamps_dec.txt $OUT/pq_stamps_enc.txt
fi
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1 || true
head -80 $OUT/summary.txt
exit 0
