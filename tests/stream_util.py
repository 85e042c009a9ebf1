"""Loader of tests/golden/stream_rsencode.npz (the reference rsencode's streams)."""
import json
import os

import numpy as np

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "stream_rsencode.npz")


def cases():
    f = np.load(FIXTURE)
    meta = json.loads(f["meta"].tobytes().decode())
    out = []
    for i, m in enumerate(meta):
        c = dict(m)
        for k in ("in", "enc", "bad", "dec"):
            c[k] = f[f"c{i}_{k}"].tobytes()
        out.append(c)
    return out


def case_ids():
    return [c["name"] for c in cases()]
