#!/bin/bash
# r05fs: FETCH_SIZE / WRITE_SIZE of tools/micro/fetch_scatter (scattered-access calibration), one
# counter per rocprofv3 run.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05fs; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 $GRAFT_REPO_ROOT/tools/micro/fetch_scatter > $OUT/plain.txt 2>&1 || { echo "plain run failed"; cat $OUT/plain.txt; exit 1; }
cat $OUT/plain.txt
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 150 timeout -s KILL 140 rocprofv3 --pmc $grp --output-format csv -d $OUT/$grp -o run -- $GRAFT_REPO_ROOT/tools/micro/fetch_scatter > $OUT/pmc_$grp.log 2>&1
  rc=$?; echo "pmc $grp rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/pmc_$grp.log; exit $rc; }
done
python3 - <<'PY'
import csv, collections, os
OUT = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r05fs"
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f"{OUT}/{c}/run_counter_collection.csv")):
        per[(r["Kernel_Name"].split("(")[0], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (k, d), v in sorted(per.items(), key=lambda x: int(x[0][1])):
        print(f"{c:10s} {k[:40]:40s} {v * 1024 / 1e6:10.1f} MB")
PY
exit 0
