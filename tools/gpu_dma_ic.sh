#!/bin/bash
# DMA-pattern probe + instruction-cache counters over a short bench run.
set -u
OUT=gpurun_out/dma; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 tools/micro/dma_patterns > $OUT/dma.log 2>&1 || exit 1
cat $OUT/dma.log
timeout -k 10 180 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH_LEVEL --output-format csv -d $OUT/p1 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/ic.log 2>&1 || exit 1
python tools/pmc_summary.py $OUT
