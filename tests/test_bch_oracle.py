"""CPU tests of the BCH restatement (oracle/ezbch_oracle.c) against the reference's own BCH fixtures:
the README vector (README.org:1173-1188), the Itron SCM captures (bch_itron.txt and
bch_itron.kelowna.txt via tests/golden/bch_itron.npz; generator asserted at bch_itron.C:225-227),
the BCH(255,k,t) shape table (swig/python/BCH/BCH.i:83-90) and init_bch's parameter limits
(bch_base:49-69).  The Djelic sources are absent from the reference (empty submodule), so these
fixtures are the whole pin; the round trips below check the restatement's self-consistency."""
import os

import numpy as np
import pytest

import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bch_itron.npz")


def _poly_int(coefs):
    return sum(int(c) << i for i, c in enumerate(coefs))


def _flip_msb_first(buf, bits):
    """Flip codeword bits counted MSB first from the start of the data (ECC bytes follow)."""
    for p in bits:
        buf[p // 8] ^= 0x80 >> (p % 8)


def _reported(bits):
    """decode_bch's location of MSB-first bit p: data[e/8] bit e%8 (bch_base:119-123)."""
    return sorted(int((p & ~7) | (7 - (p & 7))) for p in bits)


@pytest.mark.parametrize("t", range(1, 9))
def test_shape_table_m8(t):
    # BCH.i:83-90: BCH( 255, 255-8t, t ); ECC = 8t / t
    b = O.BCH(8, t)
    assert (b.n, b.n - b.ecc_bits, b.t, b.ecc_bits, b.ecc_bytes) == (255, 255 - 8 * t, t, 8 * t, t)


def test_itron_generator():
    assert _poly_int(O.BCH(8, 2).genpoly()) == 0x16F63      # bch_itron.C:225-227


def test_c5_codec_shape():
    b = O.BCH(10, 4)
    assert (b.n, b.n - b.ecc_bits, b.t, b.ecc_bytes, b.max_len) == (1023, 983, 4, 5, 122)
    # lcm of the minimal polynomials of a, a^3, a^5, a^7 over GF(2^10)/0x409
    assert _poly_int(b.genpoly()) == 0x182EBE91E9B


def test_readme_vector():
    b = O.BCH(8, 2)
    data = np.array([0x01, 0x23, 0x45, 0x67, 0x89, 0xAB, 0xCD, 0xEF], np.uint8)
    ecc = b.encode(data)
    assert ecc.tolist() == [0xCB, 0xBB]
    bad = data.copy()
    bad[1] ^= 1 << 3
    r, loc = b.correct(bad, ecc.copy())
    assert r == 1 and loc.tolist() == [11]
    np.testing.assert_array_equal(bad, data)


def test_itron_records():
    with np.load(GOLD) as z:
        msg, valid = z["msg"], z["valid"]
    assert valid.sum() == 44
    b = O.BCH(8, 2)
    for m in msg[valid]:
        assert b.encode(m[2:10]).tolist() == m[10:12].tolist()
        d, e = m[2:10].copy(), m[10:12].copy()
        assert b.correct(d, e)[0] == 0
    nfixed = 0
    for m in msg[~valid]:
        assert b.encode(m[2:10]).tolist() != m[10:12].tolist()   # none of the rejected ones is clean
        d, e = m[2:10].copy(), m[10:12].copy()
        r, loc = b.correct(d, e)
        assert r == -74 or 1 <= r <= 2
        if r > 0:
            nfixed += 1
            assert b.encode(d).tolist() == e.tolist()
            assert np.unpackbits(np.concatenate([d, e]) ^ m[2:12]).sum() == r
            assert loc.tolist() == sorted(loc.tolist())
    assert nfixed > 0


@pytest.mark.parametrize("m,t,poly", [(4, 1, 0), (16, 1, 0), (5, 0, 0), (5, 7, 0), (8, 32, 0),
                                      (8, 2, 0x101), (8, 2, 0x21d)])
def test_init_limits(m, t, poly):
    with pytest.raises(ValueError):
        O.BCH(m, t, poly)


def test_default_polynomials():
    # init_bch's defaults differ from ezpwd's RS polynomials at m = 7 and m = 14
    assert [O.BCH(m, 1).poly for m in range(5, 16)] == [
        0x25, 0x43, 0x83, 0x11D, 0x211, 0x409, 0x805, 0x1053, 0x201B, 0x402B, 0x8003]


def test_too_long_is_einval():
    b = O.BCH(10, 4)
    d = np.zeros(b.max_len + 1, np.uint8)
    assert b.correct(d, np.zeros(b.ecc_bytes, np.uint8))[0] == -22


@pytest.mark.parametrize("m,t", [(5, 2), (8, 2), (10, 4), (13, 4), (11, 5), (8, 8)])
def test_round_trips(m, t):
    b = O.BCH(m, t)
    rng = np.random.default_rng(100 * m + t)
    L = min(b.max_len, 160)
    nbits = 8 * L + b.ecc_bits
    for trial in range(40):
        data = rng.integers(0, 256, L, dtype=np.uint8)
        cw = np.concatenate([data, b.encode(data)])
        ne = trial % (t + 1)
        bits = rng.choice(nbits, ne, replace=False)
        bad = cw.copy()
        _flip_msb_first(bad, bits)
        d, e = bad[:L].copy(), bad[L:].copy()
        r, loc = b.correct(d, e)
        assert r == ne
        assert loc.tolist() == _reported(bits)
        np.testing.assert_array_equal(np.concatenate([d, e]), cw)


def test_unused_ecc_bits_are_ignored():
    b = O.BCH(5, 2)                       # 10 ECC bits in 2 bytes: 6 unused
    assert (b.ecc_bits, b.ecc_bytes) == (10, 2)
    data = np.array([0x5A], np.uint8)
    ecc = b.encode(data)
    assert ecc[1] & 0x3F == 0
    e = ecc.copy()
    e[1] ^= 0x01
    assert b.correct(data.copy(), e)[0] == 0


def test_batch_forms_match_single():
    b = O.BCH(10, 4)
    rng = np.random.default_rng(5)
    L = b.max_len
    rows = rng.integers(0, 256, (64, L + b.ecc_bytes), dtype=np.uint8)
    b.encode_batch(rows, L, nthreads=2)
    for k in range(0, 64, 9):
        assert rows[k, L:].tolist() == b.encode(rows[k, :L]).tolist()
    bad = rows.copy()
    for k in range(64):
        _flip_msb_first(bad[k], rng.choice(8 * L + b.ecc_bits, k % 6, replace=False))
    loc = np.zeros((64, 8), np.uint32)
    res = b.decode_batch(bad, L, errloc=loc, nthreads=2)
    for k in range(64):
        if k % 6 <= 4:
            assert res[k] == k % 6
            np.testing.assert_array_equal(bad[k], rows[k])
        else:
            assert res[k] == -74 or 1 <= res[k] <= 4   # 5 flips: beyond t
