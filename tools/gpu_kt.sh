#!/bin/bash
# Kernel-trace statistics of a short bench run (default library, or EZRS_LIB_VARIANT).
# Usage: tools/gpu_kt.sh <tag> [extra bench args...]
set -u
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > $OUT/kt.log 2>&1 \
    || { echo "kt failed"; tail -5 $OUT/kt.log; exit 1; }
f=$(find $OUT/kt -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f'{r["Name"][:90]:90s} calls {int(r["Calls"]):6d} avg_us {float(r["AverageNs"])/1e3:9.2f}')
EOF
exit 0
