#!/bin/bash
# Quick GPU probe: the post-synchronize step ramp (tools/step_probe.py), the short C2 bench line,
# and one PMC pass with the clock counter (GRBM_GUI_ACTIVE / 8 / kernel time = effective clock).
# Every GPU step has its own time limit; the first failure ends the script.
# Usage: tools/gpu_probe.sh <tag>
set -u
TAG=${1:-probe}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/step_probe.py 60 > $OUT/step_probe.txt 2>&1 || { echo "probe failed"; tail -5 $OUT/step_probe.txt; exit 1; }
cat $OUT/step_probe.txt
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
tail -c 600 $OUT/bench.json
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > $OUT/kt.log 2>&1 || { echo "kt failed"; tail -5 $OUT/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/clk -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > $OUT/clk.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/clk.log; exit 1; }
find $OUT -name "*.csv" | head
exit 0
