#!/bin/bash
# Ablation timings of the bit-sliced kernels (each variant under its own time limit).
set -u
OUT=gpurun_out/ablate; mkdir -p $OUT; : > $OUT/ablate.log
for v in ${ABLATE:-full nodma nocomp notr computeonly}; do
  timeout -k 10 60 tools/micro/bs_ablate_$v $v >> $OUT/ablate.log 2>&1 || { echo "ablate $v failed rc=$?"; cat $OUT/ablate.log; exit 1; }
done
cat $OUT/ablate.log
