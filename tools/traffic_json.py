#!/usr/bin/env python3
"""Build profiles/traffic.json (HBM bytes per API call per launch, read by bench.py's roofline
'traffic') from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

    python tools/traffic_json.py c2:1048576=gpurun_out/c2prof c4:65536=gpurun_out/c4prof [c5:...]

Per kernel: bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB units), the gfx950 correction of
MI355X_MICROARCH.md ("FETCH_SIZE reports exactly 1/2 of the bytes of a wide coalesced streaming
read"), which this repository calibrated on known byte counts with tools/micro/ps_stream2
(profiles/r02/fetch_calibration.json): linear 1-KiB LDS-DMA tiles read back exactly 0.50 x the span.
A call's traffic is the sum over the kernels it launches."""
import collections
import csv
import glob
import json
import os
import sys

CALLS = {
    "ezrs_encode": ("k_py_syndromes<", "true>", "k_ps_parity", "k_wide_rem", "k_wide_finish<true>"),
    "ezrs_decode": ("k_py_syndromes<", "false>", "k_decode_errors", "k_wide_rem", "k_wide_finish<false>",
                    "k_wide_errors"),
    "ezbch_encode": ("k_bch_encode", "k_bch_ps<"),
    "ezbch_decode": ("k_bch_decode", "k_bch_ps_decode"),
}


def kernel_call(name):
    for kn in ("k_pt_lin<", "k_pq_lin<"):        # k_pt_lin / k_pq_lin<codec, ENC, SH, LO0>
        if kn in name:
            return "ezrs_encode" if name.split(kn)[1].split(",")[1].strip() == "true" else "ezrs_decode"
    if "k_py_syndromes" in name or "k_pg_syndromes" in name:
        return "ezrs_encode" if "true>" in name else "ezrs_decode"
    if "k_bch_ps_decode" in name:
        return "ezbch_decode"
    if "k_bch_ps<" in name:
        return "ezbch_encode"
    for call, keys in (("ezrs_encode", ("k_ps_parity", "k_wide_finish<true>")),
                       ("ezrs_decode", ("k_decode_errors", "k_wide_finish<false>", "k_wide_errors")),
                       ("ezbch_encode", ("k_bch_encode",)), ("ezbch_decode", ("k_bch_decode",))):
        if any(k in name for k in keys):
            return call
    if "k_wide_rem" in name:
        return "rem"      # launched by both calls: counted for each
    return None


def per_kernel(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for fn in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(fn)):
            per[(r["Kernel_Name"], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        for (k, _), cs in per.items():
            for c, v in cs.items():
                acc[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    out = {"_note": __doc__.split("\n\n")[0] + " Source passes: " + " ".join(sys.argv[1:])}
    for arg in sys.argv[1:]:
        wl, d = arg.split("=", 1)
        wl, ncw = wl.split(":")
        calls = collections.defaultdict(lambda: {"hbm_bytes_per_launch": 0.0, "kernels": {}})
        rem = None
        for k, cs in per_kernel(d).items():
            if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
                continue
            call = kernel_call(k)
            if call is None:
                continue
            b = (2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024
            short = k.replace("(anonymous namespace)::", "").split("(")[0]
            if call == "rem":
                rem = (short, b)
                continue
            calls[call]["hbm_bytes_per_launch"] += b
            calls[call]["kernels"][short] = b
        if rem:
            for call in ("ezrs_encode", "ezrs_decode"):
                if call in calls:
                    calls[call]["hbm_bytes_per_launch"] += rem[1]
                    calls[call]["kernels"][rem[0]] = rem[1]
        out[wl] = {"codewords": int(ncw), **calls}
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
