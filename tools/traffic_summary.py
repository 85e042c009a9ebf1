#!/usr/bin/env python3
"""Per-kernel FETCH_SIZE / WRITE_SIZE summary of one workload's rocprofv3 --pmc passes (one counter
per run, <dir>/<counter>/run_counter_collection.csv): MB per launch (KiB x 1024 / 1e6) and traffic =
2 x FETCH + WRITE (the gfx950 correction of tools/traffic_json.py).
Usage: traffic_summary.py <pmc dir>"""
import collections
import csv
import os
import sys

d = sys.argv[1]
print(f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one counter per run ({d}); MB per launch; "
      "traffic = 2 x FETCH + WRITE")
res = collections.defaultdict(dict)
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(os.path.join(d, c, "run_counter_collection.csv"))):
        per[(r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0], r["Dispatch_Id"])] += \
            float(r["Counter_Value"])
    acc = collections.defaultdict(list)
    for (k, _), v in per.items():
        acc[k].append(v * 1024 / 1e6)
    for k, v in acc.items():
        res[k][c] = v
for k, v in res.items():
    if not ("ezrs" in k or "bch" in k) or len(v) < 2:
        continue
    f = sum(v["FETCH_SIZE"]) / len(v["FETCH_SIZE"])
    w = sum(v["WRITE_SIZE"]) / len(v["WRITE_SIZE"])
    print(f"{k[:80]:80s} launches {len(v['FETCH_SIZE'])}  FETCH {f:8.1f}  WRITE {w:8.1f}  traffic {2 * f + w:8.1f}")
