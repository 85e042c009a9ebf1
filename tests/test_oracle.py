"""CPU tests: the restatement (oracle/) against the reference's golden vectors and, where the
compiled reference (oracle/_ref) is present, against the reference itself on fresh random
trials.  No GPU needed."""
import numpy as np
import pytest

import oracle as O
from golden_util import fixture_files, fixture_id, load


@pytest.mark.parametrize("fn", fixture_files(), ids=fixture_id)
def test_restatement_matches_golden(fn):
    f = load(fn)
    mm, poly, fcr, prim, nroots, dual = (int(x) for x in f["params"])
    c = O.Codec(mm, poly, fcr, prim, nroots, bool(dual))
    T = len(f["length"])
    for t in range(T):
        L = int(f["length"][t])
        r, par = c.encode(f["enc_data"][t, :L])
        assert r == f["enc_result"][t]
        np.testing.assert_array_equal(par, f["enc_parity"][t])
        d = f["dec_data_in"][t, :L].copy()
        p = f["dec_parity_in"][t].copy()
        corr = f["dec_corr_in"][t].copy()
        ne = int(f["dec_neras"][t])
        r, pos = c.decode(d, p, f["dec_eras"][t, :ne].tolist(), corr)
        assert r == f["dec_result"][t], (t, r)
        np.testing.assert_array_equal(pos, f["dec_positions"][t, :max(r, 0)])
        np.testing.assert_array_equal(d, f["dec_data_out"][t, :L])
        np.testing.assert_array_equal(p, f["dec_parity_out"][t])
        np.testing.assert_array_equal(corr, f["dec_corr_out"][t])


def test_golden_covers_edge_regimes():
    """The fixtures must exercise clean, corrected and failed (-1) decodes."""
    seen = set()
    for fn in fixture_files():
        r = load(fn)["dec_result"]
        seen |= {"fail" if x < 0 else "clean" if x == 0 else "fixed" for x in r.tolist()}
    assert seen == {"fail", "clean", "fixed"}


def test_dual_tables_match_reference():
    if not O.Ref.available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    a, b = O.Ref.dual_tables()
    x, y = O.dual_tables()
    np.testing.assert_array_equal(a, x)
    np.testing.assert_array_equal(b, y)


def test_codec_parameter_validation():
    with pytest.raises(ValueError):
        O.Codec(8, 0x11d, 1, 1, 0)            # no roots
    with pytest.raises(ValueError):
        O.Codec(8, 0x11d, 1, 1, 255)          # nroots >= NN
    with pytest.raises(ValueError):
        O.Codec(8, 0x101, 1, 1, 32)           # x^8+1 is not primitive (rs_base:623)
    with pytest.raises(ValueError):
        O.Codec(10, 0x409, 1, 1, 32, True)    # dual basis only for 8-bit symbols


def test_field_tables_and_iprim():
    c = O.Codec(*O.ccsds_params(223))
    a, i, g = c.tables()
    assert c.iprim == 116                     # 11 * 116 = 1276 = 1 + 5*255
    assert a[255] == 0 and i[0] == 255
    assert sorted(a[:255].tolist()) == list(range(1, 256))
    assert g[nroots := 32] == 0               # monic generator (index form 0 == alpha^0)


@pytest.mark.parametrize("name", ["RS(255,223)", "RS(255,251)", "RS_CCSDS(255,223)",
                                  "RS_CCSDS_CONV(255,239)", "RS(31,26)", "RS(1023,991)"])
def test_restatement_matches_reference_random(name):
    if not O.Ref.available():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    idx = O.Ref.index(name)
    params = dict((n, p) for _, n, p in O.Ref.codecs())[name]
    c = O.Codec(*params)
    rng = np.random.default_rng(7)
    ncw = 200
    L = c.load
    data = rng.integers(0, c.nn + 1, (ncw, L)).astype(c.dtype)
    p1 = np.zeros((ncw, c.nroots), c.dtype)
    p2 = np.zeros((ncw, c.nroots), c.dtype)
    O.Ref.encode_batch(idx, data, L, p1)
    c.encode_batch(data, L, p2)
    np.testing.assert_array_equal(p1, p2)
    # corrupt: up to 1.5x capacity errors, batch decode both ways
    cw1 = np.concatenate([data, p1], axis=1)
    for k in range(ncw):
        ne = int(rng.integers(0, c.nroots * 3 // 4 + 1))
        loc = rng.choice(cw1.shape[1], ne, replace=False)
        cw1[k, loc] ^= rng.integers(1, c.nn + 1, ne).astype(c.dtype)
    d1, q1 = cw1[:, :L].copy(), cw1[:, L:].copy()
    d2, q2 = d1.copy(), q1.copy()
    pos1 = np.zeros((ncw, c.nroots), np.uint32)
    pos2 = np.zeros((ncw, c.nroots), np.uint32)
    r1 = O.Ref.decode_batch(idx, d1, L, q1, positions=pos1)
    r2 = c.decode_batch(d2, L, q2, positions=pos2)
    np.testing.assert_array_equal(r1, r2)
    np.testing.assert_array_equal(d1, d2)
    np.testing.assert_array_equal(q1, q2)
    for k in range(ncw):
        np.testing.assert_array_equal(pos1[k, :max(r1[k], 0)], pos2[k, :max(r2[k], 0)])
