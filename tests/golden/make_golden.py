"""Generate the golden RS fixtures in tests/golden/*.npz FROM THE REFERENCE ITSELF.

Run in the build container (where /root/reference exists):

    make -C oracle ref && python tests/golden/make_golden.py

Every expected output below comes from oracle/_ref/libezrs_ref.so, i.e. the reference's own
ezpwd::RS<N,K> / RS_CCSDS / RS_CCSDS_CONV templates (c++/ezpwd/rs:74-104) compiled from the
unmodified headers, called through encode<INP>(data,len,parity) (rs_base:868-904) and
decode<INP>(data,len,parity,eras_pos,no_eras,corr) (rs_base:1170-1242).  The fixture files hold
data only (inputs and the reference's outputs); no reference source is stored.

Trial mix per codec (mirrors exercise.H:100-178 and rsvalidate.C:130-206): random shortened
payload lengths, error+erasure loads from 0 to 3x the correction capacity (so the overwhelmed
regime -- result -1, partial in-place corrections -- is covered), erasures that are not
actually corrupted, duplicated erasures, out-of-range erasures, and (for masked codecs) junk bits
above the symbol width in data and parity.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402


def trials_for(nn):
    if nn <= 255:
        return 48
    if nn <= 1023:
        return 12
    return 4


def main():
    if not O.Ref.available():
        raise SystemExit("oracle/_ref/libezrs_ref.so missing: run `make -C oracle ref` first")
    rng = np.random.default_rng(0x5EED0001)
    for idx, name, params in O.Ref.codecs():
        mm, poly, fcr, prim, nroots, dual = params
        nn = (1 << mm) - 1
        load = nn - nroots
        dt = np.uint8 if mm <= 8 else np.uint16
        width_hi = 1 << (8 * np.dtype(dt).itemsize)
        T = trials_for(nn)
        maxlen = min(load, 400)  # keep the wide-symbol fixtures small: shortened codewords
        E = nroots + 2
        f = dict(params=np.array([mm, poly, fcr, prim, nroots, int(dual)], np.int64),
                 length=np.zeros(T, np.int32),
                 enc_data=np.zeros((T, maxlen), dt), enc_parity=np.zeros((T, nroots), dt),
                 enc_result=np.zeros(T, np.int32),
                 dec_data_in=np.zeros((T, maxlen), dt), dec_parity_in=np.zeros((T, nroots), dt),
                 dec_neras=np.zeros(T, np.int32), dec_eras=np.zeros((T, E), np.uint32),
                 dec_corr_in=np.zeros((T, nroots), dt),
                 dec_result=np.zeros(T, np.int32), dec_positions=np.zeros((T, nroots), np.uint32),
                 dec_data_out=np.zeros((T, maxlen), dt), dec_parity_out=np.zeros((T, nroots), dt),
                 dec_corr_out=np.zeros((T, nroots), dt))
        for t in range(T):
            L = int(rng.integers(1, maxlen + 1)) if t % 4 else maxlen
            junk = (t % 7 == 3) and mm < 8 * np.dtype(dt).itemsize
            data = rng.integers(0, width_hi if junk else nn + 1, L).astype(dt)
            r, par = O.Ref.encode(idx, data, nroots, dt)
            f["length"][t] = L
            f["enc_data"][t, :L] = data
            f["enc_parity"][t] = par
            f["enc_result"][t] = r
            cw = np.concatenate([data & nn, par]).astype(dt)
            n = L + nroots
            tee = int(nroots * [0.0, 0.25, 0.5, 0.75, 1.0, 1.0, 1.25, 2.0, 3.0][t % 9])
            ne = nera = 0
            eras = []
            locs = rng.permutation(n)
            i = 0
            while 2 * ne + nera + 1 <= tee and i < n:
                loc = int(locs[i]); i += 1
                v = int(rng.integers(1, nn + 1))
                if rng.random() < 0.5 and nera < nroots:
                    eras.append(loc); nera += 1
                    if rng.random() < 0.85:
                        cw[loc] ^= v
                else:
                    ne += 1
                    cw[loc] ^= v
            if t % 11 == 5 and eras:
                eras.append(eras[0])
            if t % 13 == 6:
                eras.append(n + 1)
            eras = eras[:nroots]
            if junk:
                cw[:L] |= dt((t * 0x35) & (width_hi - 1) & ~nn)
                if t % 2:
                    cw[L] |= dt(1 << mm)
            d, p = cw[:L].copy(), cw[L:].copy()
            corr = rng.integers(0, nn + 1, nroots).astype(dt)
            f["dec_data_in"][t, :L] = d
            f["dec_parity_in"][t] = p
            f["dec_neras"][t] = len(eras)
            f["dec_eras"][t, :len(eras)] = eras
            f["dec_corr_in"][t] = corr
            r, pos = O.Ref.decode(idx, d, p, nroots, eras, corr)
            f["dec_result"][t] = r
            f["dec_positions"][t, :len(pos)] = pos
            f["dec_data_out"][t, :L] = d
            f["dec_parity_out"][t] = p
            f["dec_corr_out"][t] = corr
        fn = os.path.join(HERE, "rs_" + name.replace("(", "_").replace(",", "_").replace(")", "")
                          + ".npz")
        np.savez_compressed(fn, **f)
        print(f"{name:24s} {T:3d} trials  results {sorted(set(f['dec_result'].tolist()))[:8]}")


if __name__ == "__main__":
    main()
