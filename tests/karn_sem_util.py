"""Shared loader of tests/golden/karn_sem.npz (tests/golden/make_karn_sem_fixtures.py): libfec's own
outputs for the Karn-semantics cases (shortened codes, full-frame positions, overwhelmed words)."""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
KINDS = ("char", "int", "8", "ccsds")


def cases():
    f = np.load(os.path.join(HERE, "golden", "karn_sem.npz"))
    out = []
    for ci in range(int(f["ncases"][0])):
        pre = f"c{ci}_"
        meta = f[pre + "meta"]
        c = {k: f[pre + k] for k in ("data", "parity", "dec_in", "dec_eras", "dec_neras", "dec_result",
                                    "dec_out", "dec_positions")}
        c["kind"] = KINDS[int(meta[0])]
        c["params"] = tuple(int(x) for x in meta[1:6])
        c["pad"] = int(meta[6])
        c["id"] = f"{c['kind']}-m{c['params'][0]}-nr{c['params'][4]}-pad{c['pad']}"
        out.append(c)
    return out
