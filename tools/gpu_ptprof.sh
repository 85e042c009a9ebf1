#!/bin/bash
# Tile-kernel study: phase ablations (timing only), the pair-kernel A/B, and PMC groups of the C2 bench.
# Usage: tools/gpu_ptprof.sh <tag>
set -u
TAG=$1; OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 180 python tools/pt_ablate.py 0 1 2 4 8 3 > $OUT/ablate.log 2>&1 || { echo "ablate failed"; tail -5 $OUT/ablate.log; exit 1; }
cat $OUT/ablate.log
EZRS_PS_VARIANT=pair timeout -k 10 120 python tools/pt_ablate.py 0 > $OUT/ablate_pair.log 2>&1 || { echo "pair failed"; tail -5 $OUT/ablate_pair.log; exit 1; }
cat $OUT/ablate_pair.log
bash tools/gpu_prof.sh $TAG/prof
python3 tools/pmc_summary.py $OUT/prof > $OUT/pmc_summary.txt 2>&1; head -c 6000 $OUT/pmc_summary.txt
