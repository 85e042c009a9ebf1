#!/bin/bash
# r05q: kernel traces of the shard sweep points (1 KiB, 1 MiB) and C5 decode phase ablations.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05q; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-extras"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shards -o run -- python3 $GRAFT_REPO_ROOT/tools/shard_time.py 1024 50 > $OUT/prof_shards.log 2>&1 || { echo "prof shards failed"; tail -5 $OUT/prof_shards.log; exit 1; }
tail -1 $OUT/prof_shards.log
python3 - <<'PY'
import csv, os
d = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r05q/prof_shards/run_kernel_stats.csv"
for r in csv.DictReader(open(d)):
    print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "us")
PY
exit 0
