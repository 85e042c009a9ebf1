"""Generate the Karn-side golden vectors tests/golden/karn_*.npz FROM PHIL KARN'S LIBFEC ITSELF.

Run in the build container (where /root/reference exists):

    make -C oracle karn && python tests/golden/make_karn_fixtures.py

Every expected output comes from oracle/_ref/libkarn.so: fec-3.0.1's encode_rs_char /
decode_rs_char (the general codec of phil-karn/rstest.c's Tab, row {8,0x11d,1,1,32} = BASELINE
config C2), encode_rs_8 / decode_rs_8 (the fixed CCSDS-polynomial codec in the conventional basis)
and encode_rs_ccsds / decode_rs_ccsds (dual basis), compiled from the unmodified tarball sources.
The files hold data only: inputs and libfec's outputs.

Trial mix: full-length codewords (pad 0, where Karn's and ezpwd's error positions coincide:
fec-3.0.1/decode_rs.h:114,295 vs rs_base:1440-1442), e errors and f erasures with 2e + f <= nroots
(libfec and ezpwd agree on every decodable word; beyond capacity ezpwd adds failure checks that
libfec lacks, rsvalidate.C:290-296), erasures that are not actually corrupted included.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402

NCW = 1024
NR = 32
K = 255 - NR


def corrupt(rng, cw):
    """Errors + erasures within capacity; returns (rows, eras [ncw, NR] int32, neras)."""
    ncw = cw.shape[0]
    rows = cw.copy()
    eras = np.zeros((ncw, NR), np.int32)
    neras = np.zeros(ncw, np.int32)
    for i in range(ncw):
        f = int(rng.integers(0, NR + 1)) if i % 3 else 0          # erasures
        e = int(rng.integers(0, (NR - f) // 2 + 1))               # errors
        locs = rng.choice(255, e + f, replace=False)
        flip = rng.integers(1, 256, e + f).astype(np.uint8)
        # a quarter of the erasures are not corrupted (rstest/exercise.c:189-210 style)
        keep = rng.random(e + f) < 0.25
        keep[:e] = False                                          # errors always corrupt
        flip[keep] = 0
        rows[i, locs] ^= flip
        eras[i, :f] = locs[e:]
        neras[i] = f
    return rows, eras, neras


def main():
    if not O.Karn.available():
        raise SystemExit("oracle/_ref/libkarn.so missing: run `make -C oracle karn` first")
    rng = np.random.default_rng(0x4B41524E)
    # general char codec {8, 0x11d, fcr 1, prim 1, 32} (= ezpwd::RS<255,223>)
    params = (8, 0x11d, 1, 1, NR, 0)
    data = rng.integers(0, 256, (NCW, K)).astype(np.uint8)
    par = O.Karn.encode_char(params, data, K)
    cw = np.concatenate([data, par], axis=1)
    rows, eras, neras = corrupt(rng, cw)
    out = rows.copy()
    pos = eras.copy()
    res = O.Karn.decode_char(params, out, pos, neras)
    np.savez_compressed(os.path.join(HERE, "karn_rs255_223.npz"), params=np.array(params[:5], np.int64),
                        data=data, parity=par, dec_in=rows, dec_eras=eras, dec_neras=neras,
                        dec_result=res, dec_out=out, dec_positions=pos)
    assert (res >= 0).all() and (out == cw).all(), "libfec failed inside capacity?"
    # fixed CCSDS codecs: conventional basis (encode_rs_8) and dual basis (encode_rs_ccsds)
    for kind in ("8", "ccsds"):
        data = rng.integers(0, 256, (NCW, K)).astype(np.uint8)
        par = O.Karn.encode_fixed(kind, data)
        cw = np.concatenate([data, par], axis=1)
        rows, eras, neras = corrupt(rng, cw)
        out = rows.copy()
        pos = eras.copy()
        res = O.Karn.decode_fixed(kind, out, pos, neras)
        assert (res >= 0).all() and (out == cw).all(), "libfec failed inside capacity?"
        np.savez_compressed(os.path.join(HERE, f"karn_{kind}.npz"), data=data, parity=par, dec_in=rows,
                            dec_eras=eras, dec_neras=neras, dec_result=res, dec_out=out, dec_positions=pos)
    print("karn fixtures written")


if __name__ == "__main__":
    main()
