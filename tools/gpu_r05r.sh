#!/bin/bash
# r05r: kernel traces of the 1 MiB shard point and of a plain C2 batch of the same codeword count.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05r; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
summ() {
python3 - "$1" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "ezrs" in r["Name"]:
        print("  ", r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1000, 1), "us")
PY
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_1m -o run -- python3 $GRAFT_REPO_ROOT/tools/shard_time.py 1048576 50 > $OUT/prof_1m.log 2>&1 || { echo "prof 1m failed"; tail -5 $OUT/prof_1m.log; exit 1; }
tail -1 $OUT/prof_1m.log; summ $OUT/prof_1m/run_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-extras --ncw 1203968 --steps 50 --warmup 5 --spinup 0.1 > $OUT/prof_c2.log 2>&1 || { echo "prof c2 failed"; tail -5 $OUT/prof_c2.log; exit 1; }
summ $OUT/prof_c2/run_kernel_stats.csv
exit 0
