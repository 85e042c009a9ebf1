#!/usr/bin/env python3
"""Extract the reference's BCH fixtures into tests/golden/bch_itron.npz (data only).

Source: the Itron SCM radio captures shipped with the reference, bch_itron.txt and
bch_itron.kelowna.txt, one record per line as "<96 bits> : <description>" (read by
bch_itron.C:144-177).  Each record is a 12-byte message: bytes 2..9 are the BCH(255,239,2) payload
and bytes 10..11 its 16 ECC bits (bch_itron.C:167-177).  Lines whose description starts with
"{Time:" were accepted by the capture tool; "Bad CRC" lines were not.  Run where /root/reference
exists; the tests only read the .npz.
"""
import os
import sys

import numpy as np

REF = os.environ.get("EZPWD_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bch_itron.npz")
FILES = ("bch_itron.txt", "bch_itron.kelowna.txt")


def parse(path):
    msgs, valid = [], []
    with open(path) as f:
        for line in f:
            bits, sep, desc = line.partition(":")
            bits = bits.strip()
            if not sep or len(bits) != 96 or set(bits) - {"0", "1"}:
                continue
            msgs.append([int(bits[8 * i:8 * i + 8], 2) for i in range(12)])
            valid.append(desc.strip().startswith("{Time:"))
    return msgs, valid


def main():
    msgs, valid, src = [], [], []
    for i, fn in enumerate(FILES):
        m, v = parse(os.path.join(REF, fn))
        msgs += m
        valid += v
        src += [i] * len(m)
    np.savez_compressed(OUT, msg=np.array(msgs, np.uint8), valid=np.array(valid, bool),
                        source=np.array(src, np.uint8))
    print(f"{OUT}: {len(msgs)} records, {sum(valid)} valid")
    return 0


if __name__ == "__main__":
    sys.exit(main())
