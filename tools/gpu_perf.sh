#!/bin/bash
# Perf-analysis session: ablation timings, PMC passes over the bench, FETCH_SIZE calibration on the
# DMA-pattern probe.  Every GPU step has its own time limit; any failure stops the script.
# Usage: tools/gpu_perf.sh <tag>
set -u
TAG=${1:-perf}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for v in full nodma nocomp notr; do
  timeout -k 10 60 tools/micro/bs_ablate_$v $v >> $OUT/ablate.log 2>&1 || { echo "ablate $v failed rc=$?"; exit 1; }
done
cat $OUT/ablate.log
bash tools/pmc.sh $TAG/pmc || exit 1
python tools/pmc_summary.py gpurun_out/$TAG/pmc $OUT/pmc_summary.json > $OUT/pmc_summary.txt || exit 1
bash tools/pmc_cmd.sh $TAG/cal "FETCH_SIZE" "WRITE_SIZE" -- tools/micro/dma_patterns || exit 1
python tools/pmc_summary.py gpurun_out/$TAG/cal --all > $OUT/cal_summary.txt 2>&1 || true
exit 0
