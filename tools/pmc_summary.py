#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (tools/pmc.sh output): per kernel, the average per dispatch of
each counter.  HBM traffic per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB units in rocprofv3),
applying the gfx950 correction from MI355X_MICROARCH.md ("FETCH_SIZE reports exactly 1/2 of the
bytes of a wide coalesced streaming read")."""
import collections
import csv
import glob
import json
import os
import sys


def load(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for fn in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(fn)):
            k = r["Kernel_Name"]
            per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        for (k, _), cs in per.items():
            for c, v in cs.items():
                acc[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    keep_all = "--all" in sys.argv
    d = args[0]
    res = load(d)
    out = {}
    for k, cs in res.items():
        if "ezrs" not in k and "bch" not in k and not keep_all:
            continue
        short = k.replace("(anonymous namespace)::", "").split("(")[0][-60:]
        o = dict(cs)
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            o["hbm_bytes_per_launch"] = (2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024
            o["fetch_bytes_raw"] = cs["FETCH_SIZE"] * 1024
            o["write_bytes"] = cs["WRITE_SIZE"] * 1024
        out[short] = o
        print(short)
        for c in sorted(o):
            print(f"   {c:28s} {o[c]:.6g}")
    if len(args) > 1:
        json.dump(out, open(args[1], "w"), indent=1)


if __name__ == "__main__":
    main()
