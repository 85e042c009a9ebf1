"""Generate tests/golden/karn_sem.npz FROM PHIL KARN'S LIBFEC ITSELF: the Karn-semantics vectors for
the Karn ABI over the engine (include/ezrs_fec.h, EZRS_SEM_KARN).

Run in the build container (where /root/reference exists):

    make -C oracle karn && python tests/golden/make_karn_sem_fixtures.py

Every expected output comes from oracle/_ref/libkarn.so (fec-3.0.1 compiled from the reference's
tarball with its int-symbol patch): init/encode/decode_rs_char, init/encode/decode_rs_int,
encode/decode_rs_8, encode/decode_rs_ccsds.  Unlike tests/golden/karn_*.npz (pad 0, inside capacity,
where Karn and ezpwd agree) these cases exercise what differs:
  * shortened codewords (pad > 0): erasure and corrected positions in the full NN frame
    (fec-3.0.1/decode_rs.h:114, 295), erasures inside the pad included;
  * loads up to 1.6x the parity: overwhelmed words where libfec returns a count where ezpwd returns
    -1 (deg lambda = 0, a zero Forney denominator, a root in the pad: decode_rs.h:232-289);
  * rstest.c's Tab codecs of every symbol size (phil-karn/rstest.c:26-50), int symbols for m > 8.
The file holds data only: inputs and libfec's outputs.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402

# (kind, (symsize, gfpoly, fcr, prim, nroots), pad, ncw)
CASES = [
    ("char", (8, 0x11d, 1, 1, 32), 0, 384),
    ("char", (8, 0x11d, 1, 1, 32), 61, 384),
    ("char", (8, 0x11d, 1, 1, 16), 150, 256),
    ("char", (8, 0x11d, 1, 1, 4), 200, 256),
    ("char", (8, 0x187, 112, 11, 16), 40, 256),
    ("char", (8, 0x187, 112, 11, 64), 10, 128),
    ("char", (2, 0x7, 1, 1, 1), 0, 256),
    ("char", (3, 0xb, 1, 1, 2), 1, 256),
    ("char", (4, 0x13, 1, 1, 4), 3, 256),
    ("char", (5, 0x25, 1, 1, 6), 7, 256),
    ("char", (6, 0x43, 1, 1, 8), 20, 256),
    ("char", (7, 0x89, 1, 1, 10), 50, 256),
    ("int", (9, 0x211, 1, 1, 32), 300, 64),
    ("int", (10, 0x409, 1, 1, 32), 800, 64),
    ("int", (12, 0x1053, 1, 1, 32), 3900, 32),
    ("int", (16, 0x1100b, 1, 1, 32), 65535 - 32 - 180, 32),
    ("8", (8, 0x187, 112, 11, 32), 0, 256),
    ("8", (8, 0x187, 112, 11, 32), 100, 256),
    ("ccsds", (8, 0x187, 112, 11, 32), 0, 256),
    ("ccsds", (8, 0x187, 112, 11, 32), 33, 256),
]


def corrupt(rng, rows, nn, nroots, pad, m):
    """Errors in the row, erasures anywhere in the full frame (some in the pad, some repeated,
    some not corrupted); loads 0 .. 1.6 x nroots.  Returns (rows, eras int32 [ncw, nroots], neras)."""
    ncw, L = rows.shape
    out = rows.copy()
    eras = np.zeros((ncw, nroots), np.int32)
    neras = np.zeros(ncw, np.int32)
    for i in range(ncw):
        load = int(rng.integers(0, int(1.6 * nroots) + 2))
        f = min(int(rng.integers(0, load + 1)), nroots, L)
        e = min((load - f + 1) // 2, L - f)
        locs = rng.choice(L, e + f, replace=False)               # row indices (frame = pad + idx)
        vals = rng.integers(1, 1 << m, e + f).astype(out.dtype)
        keep = rng.random(e + f) < 0.2                           # erasures not actually corrupted
        keep[:e] = False
        vals[keep] = 0
        out[i, locs] ^= vals
        ep = (locs[e:] + pad).astype(np.int32)
        if f and pad and rng.random() < 0.15:                    # an erasure inside the pad
            ep[0] = int(rng.integers(0, pad))
        if f > 1 and rng.random() < 0.05:                        # a repeated erasure
            ep[1] = ep[0]
        eras[i, :f] = ep
        neras[i] = f
    return out, eras, neras


def main():
    if not O.Karn.available():
        raise SystemExit("oracle/_ref/libkarn.so missing: run `make -C oracle karn` first")
    rng = np.random.default_rng(0x4B41524F)
    arrays = {}
    for ci, (kind, p, pad, ncw) in enumerate(CASES):
        m, nr = p[0], p[4]
        nn = (1 << m) - 1
        K = nn - nr - pad
        dt = np.uint16 if kind == "int" else np.uint8
        data = rng.integers(0, 1 << m, (ncw, K)).astype(dt)
        params = p + (pad,)
        if kind == "char":
            par = O.Karn.encode_char(params, data, K)
        elif kind == "int":
            par = O.Karn.encode_int(params, data, K)
        else:
            par = O.Karn.encode_fixed(kind, data, pad)
        cw = np.concatenate([data, par], axis=1)
        rows, eras, neras = corrupt(rng, cw, nn, nr, pad, m)
        out = rows.copy()
        pos = eras.copy()
        if kind == "char":
            res = O.Karn.decode_char(params, out, pos, neras)
        elif kind == "int":
            res = O.Karn.decode_int(params, out, pos, neras)
        else:
            res = O.Karn.decode_fixed(kind, out, pos, neras, pad)
        pre = f"c{ci}_"
        arrays[pre + "meta"] = np.array([("char", "int", "8", "ccsds").index(kind)] + list(p) + [pad], np.int64)
        for k, v in (("data", data), ("parity", par), ("dec_in", rows), ("dec_eras", eras),
                     ("dec_neras", neras), ("dec_result", res), ("dec_out", out), ("dec_positions", pos)):
            arrays[pre + k] = v
        print(f"case {ci}: {kind} {p} pad {pad}: results {np.bincount(np.clip(res, -1, 99) + 1)[:6]}...")
    arrays["ncases"] = np.array([len(CASES)])
    np.savez_compressed(os.path.join(HERE, "karn_sem.npz"), **arrays)
    print("karn_sem.npz written")


if __name__ == "__main__":
    main()
