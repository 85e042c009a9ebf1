"""GF(2^16) fast path (ezrs_wide.hip: remainder networks + syndrome/parity finish + wavefront
error path) against the oracle: parity, results, corrected rows, positions and corrections, for
clean, correctable and overwhelmed codewords, with erasures, shortened lengths and batch sizes that
are not a multiple of the 128-codeword tile.  Each case also runs with EZRS_NO_WIDE=1 (the
lane-group kernels) so both device paths stay pinned to the oracle."""
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as T
    if not T.cuda.is_available():
        pytest.skip("no GPU")
    return T


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).view(torch.uint16).cuda()


def _host(t):
    import torch
    return t.cpu().view(torch.int16).numpy().view(np.uint16)


def _codec(n, k, wide):
    import ezrs
    old = os.environ.get("EZRS_NO_WIDE")
    os.environ["EZRS_NO_WIDE"] = "0" if wide else "1"
    try:
        return ezrs.Codec.rs(n, k)
    finally:
        if old is None:
            del os.environ["EZRS_NO_WIDE"]
        else:
            os.environ["EZRS_NO_WIDE"] = old


CASES = [  # n, k, ncw, L
    (65535, 65503, 300, 700),
    (65535, 65503, 129, 5000),
    (65535, 65503, 4, 65503),
    (65535, 65519, 200, 1500),
    (65535, 65503, 1, 333),
]


@pytest.mark.parametrize("wide", [True, False], ids=["wide", "lanes"])
@pytest.mark.parametrize("n,k,ncw,L", CASES)
def test_wide_vs_oracle(torch, n, k, ncw, L, wide):
    if not wide and L > 5000:
        pytest.skip("lane kernels: full length covered by test_gpu_parity")
    c = _codec(n, k, wide)
    oc = O.Codec(*O.rs_params(n, k))
    nr = n - k
    rng = np.random.default_rng(n + k + ncw + L)
    host = rng.integers(0, n + 1, (ncw, L + nr)).astype(np.uint16)
    ref = host.copy()
    oc.encode_batch(ref, L)
    # encode, inline parity
    dev = _dev(torch, host)
    c.encode(dev, L)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(dev), ref)
    # encode, separate parity buffer, data rows at a wider stride
    wdata = np.zeros((ncw, L + 7), np.uint16)
    wdata[:, :L] = ref[:, :L]
    par = torch.zeros((ncw, nr + 3), dtype=torch.uint16, device="cuda")
    c.encode(_dev(torch, wdata), L, par)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(par)[:, :nr], ref[:, L:])
    # corrupt: loads from 0 to 1.5x capacity, random erasure subsets (some erasures clean)
    cw = ref.copy()
    eras = np.zeros((ncw, nr), np.uint32)
    neras = np.zeros(ncw, np.uint32)
    for i in range(ncw):
        m = int(rng.integers(0, 3 * nr // 2 + 1)) if i % 5 else int(rng.integers(0, 3))
        m = min(m, L + nr)
        locs = rng.choice(L + nr, m, replace=False)
        cw[i, locs] ^= rng.integers(1, n + 1, m).astype(np.uint16)
        ne = min(int(rng.integers(0, m + 1)), nr)
        eras[i, :ne] = locs[:ne]
        if i % 7 == 3 and ne < nr:                 # an erasure on an uncorrupted symbol
            clean = np.setdiff1d(np.arange(L + nr), locs)
            if len(clean):
                eras[i, ne] = clean[0]
                ne += 1
        neras[i] = ne
    exp = cw.copy()
    exp_pos = np.zeros((ncw, nr), np.uint32)
    exp_r = oc.decode_batch(exp, L, None, eras, neras, exp_pos, nthreads=8)
    d = _dev(torch, cw)
    pos = torch.zeros((ncw, nr), dtype=torch.int32, device="cuda")
    r = c.decode(d, L, eras=torch.from_numpy(eras.view(np.int32)).cuda(),
                 neras=torch.from_numpy(neras.view(np.int32)).cuda(), positions=pos)
    torch.cuda.synchronize()
    r = r.cpu().numpy()
    np.testing.assert_array_equal(r, exp_r)
    np.testing.assert_array_equal(_host(d), exp)
    got = pos.cpu().numpy().view(np.uint32)
    for i in np.nonzero(r > 0)[0]:
        np.testing.assert_array_equal(got[i, :r[i]], exp_pos[i, :r[i]])
    if ncw > 4:
        assert (r == 0).any() and (r > 0).any() and (r == -1).any()


@pytest.mark.parametrize("wide", [True, False], ids=["wide", "lanes"])
def test_wide_corrections_and_bad_erasures(torch, wide):
    """corr[] output, erasure lists that the reference rejects (too many, out of range), and an
    erasure-only codeword whose syndromes are zero (result 0)."""
    n, k, L = 65535, 65503, 400
    c = _codec(n, k, wide)
    oc = O.Codec(*O.rs_params(n, k))
    nr = n - k
    rng = np.random.default_rng(5)
    ncw = 6
    ref = rng.integers(0, n + 1, (ncw, L + nr)).astype(np.uint16)
    oc.encode_batch(ref, L)
    cw = ref.copy()
    eras = np.zeros((ncw, nr), np.uint32)
    neras = np.zeros(ncw, np.uint32)
    cw[0, [3, 50, 399, 420]] ^= np.array([1, 2, 3, 4], np.uint16)       # 4 errors
    cw[1, [7, 8]] ^= np.array([9, 9], np.uint16)
    eras[1, :2] = [7, 8]
    neras[1] = 2                                                          # 2 erasures
    eras[2, :3] = [1, 2, 3]
    neras[2] = 3                                                          # clean, erasures
    eras[3, 0] = L + nr                                                   # out of range
    neras[3] = 1
    cw[4, 10] ^= 1
    neras[4] = 0
    cw[5, :40] ^= 1                                                       # overwhelmed
    d = _dev(torch, cw)
    corr = torch.zeros((ncw, nr), dtype=torch.uint16, device="cuda")
    pos = torch.zeros((ncw, nr), dtype=torch.int32, device="cuda")
    r = c.decode(d, L, eras=torch.from_numpy(eras.view(np.int32)).cuda(),
                 neras=torch.from_numpy(neras.view(np.int32)).cuda(), positions=pos, corr=corr)
    torch.cuda.synchronize()
    r = r.cpu().numpy()
    got_d, got_c = _host(d), _host(corr)
    for i in range(ncw):
        data = cw[i, :L].copy()
        par = cw[i, L:].copy()
        cc = np.zeros(nr, np.uint16)
        er, ep = oc.decode(data, par, eras[i, :neras[i]].tolist(), cc)
        assert r[i] == er, f"row {i}"
        np.testing.assert_array_equal(got_d[i, :L], data)
        np.testing.assert_array_equal(got_d[i, L:], par)
        if er > 0:
            np.testing.assert_array_equal(got_c[i, :er], cc[:er])
    assert list(r[:4]) == [4, 2, 0, -1] and r[4] == 1


def test_wide_root_finder_degrees(torch):
    """The error path's root finder (Berlekamp trace splitting, direct quadratic solve) at every
    locator degree 1..32: e errors + f erasures with 2e + f <= 32 in turn, then overwhelmed rows
    (locators that do not split over GF(2^16), or split with repeated roots), repeated erasure
    positions, erasures on the parity and on the first and last symbols."""
    n, k, L = 65535, 65503, 900
    nr = n - k
    c = _codec(n, k, True)
    oc = O.Codec(*O.rs_params(n, k))
    rng = np.random.default_rng(77)
    plan = [(e, f) for e in range(17) for f in range(nr - 2 * e + 1)]        # all correctable loads
    plan += [(e, 0) for e in range(17, 33)] * 6 + [(e, 4) for e in range(15, 30)] * 4
    ncw = len(plan) + 40
    ref = rng.integers(0, n + 1, (ncw, L + nr)).astype(np.uint16)
    oc.encode_batch(ref, L)
    cw = ref.copy()
    eras = np.zeros((ncw, nr), np.uint32)
    neras = np.zeros(ncw, np.uint32)
    for i, (e, f) in enumerate(plan):
        locs = rng.choice(L + nr, e + f, replace=False)
        if i % 3 == 0 and e + f >= 2:
            locs[0], locs[-1] = 0, L + nr - 1
        cw[i, locs] ^= rng.integers(1, n + 1, e + f).astype(np.uint16)
        f = min(f, nr)
        eras[i, :f] = locs[e:e + f]
        neras[i] = f
    for i in range(len(plan), ncw):              # repeated erasure positions, 1-3 errors
        e = 1 + i % 3
        locs = rng.choice(L + nr, e + 2, replace=False)
        cw[i, locs[:e]] ^= 1 + (i % 65535)
        eras[i, :4] = [locs[e], locs[e + 1], locs[e], L + nr - 1 - i % nr]
        neras[i] = 4
    exp = cw.copy()
    exp_pos = np.zeros((ncw, nr), np.uint32)
    exp_r = oc.decode_batch(exp, L, None, eras, neras, exp_pos, nthreads=8)
    d = _dev(torch, cw)
    pos = torch.zeros((ncw, nr), dtype=torch.int32, device="cuda")
    r = c.decode(d, L, eras=torch.from_numpy(eras.view(np.int32)).cuda(),
                 neras=torch.from_numpy(neras.view(np.int32)).cuda(), positions=pos)
    torch.cuda.synchronize()
    r = r.cpu().numpy()
    np.testing.assert_array_equal(r, exp_r)
    np.testing.assert_array_equal(_host(d), exp)
    got = pos.cpu().numpy().view(np.uint32)
    for i in np.nonzero(r > 0)[0]:
        np.testing.assert_array_equal(got[i, :r[i]], exp_pos[i, :r[i]])
    assert (r[:len(plan)][:300] > 0).sum() > 250 and (r == -1).sum() > 50


def test_wide_multi_pass_batch(torch):
    """A batch larger than one pass of the persistent finishing grid (CUs x 64 codewords) and of the
    error kernel's grid: parity against the oracle, then a decode round trip with 0..16 errors per
    codeword (result = error count, rows restored)."""
    n, k, L = 65535, 65503, 97
    nr = n - k
    ncw = 40000
    c = _codec(n, k, True)
    oc = O.Codec(*O.rs_params(n, k))
    rng = np.random.default_rng(11)
    ref = rng.integers(0, n + 1, (ncw, L + nr)).astype(np.uint16)
    oc.encode_batch(ref, L)
    h = ref.copy()
    h[:, L:] = 0
    dev = _dev(torch, h)
    c.encode(dev, L)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_host(dev), ref)
    cw = ref.copy()
    nerr = np.arange(ncw) % 17
    for i in range(ncw):
        locs = rng.choice(L + nr, nerr[i], replace=False)
        cw[i, locs] ^= rng.integers(1, n + 1, nerr[i]).astype(np.uint16)
    d = _dev(torch, cw)
    r = c.decode(d, L)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(r.cpu().numpy(), nerr)
    np.testing.assert_array_equal(_host(d), ref)


def test_wide_full_length_1k(torch):
    """C4 shape at 1024 full-length RS(65535,65503) codewords (134 MB): parity, and the decode of
    8 errors + 4 erasures in every codeword (results, corrected rows, positions), all against the
    oracle."""
    c = _codec(65535, 65503, True)
    oc = O.Codec(*O.rs_params(65535, 65503))
    ncw, L, nr = 1024, 65503, 32
    rng = np.random.default_rng(0xC4)
    host = rng.integers(0, 65536, (ncw, L + nr)).astype(np.uint16)
    dev = _dev(torch, host)
    c.encode(dev, L)
    oc.encode_batch(host, L, nthreads=16)
    np.testing.assert_array_equal(_host(dev), host)
    cw = host.copy()
    eras = np.zeros((ncw, nr), np.uint32)
    neras = np.full(ncw, 4, np.uint32)
    for i in range(ncw):
        locs = rng.choice(L + nr, 12, replace=False)
        cw[i, locs] ^= rng.integers(1, 65536, 12).astype(np.uint16)
        eras[i, :4] = locs[8:]
    exp = cw.copy()
    exp_pos = np.zeros((ncw, nr), np.uint32)
    exp_r = oc.decode_batch(exp, L, None, eras, neras, exp_pos, nthreads=16)
    d = _dev(torch, cw)
    pos = torch.zeros((ncw, nr), dtype=torch.int32, device="cuda")
    r = c.decode(d, L, eras=torch.from_numpy(eras.view(np.int32)).cuda(),
                 neras=torch.from_numpy(neras.view(np.int32)).cuda(), positions=pos)
    r = r.cpu().numpy()
    np.testing.assert_array_equal(r, exp_r)
    assert (r == 12).all()
    np.testing.assert_array_equal(_host(d), exp)
    np.testing.assert_array_equal(_host(d), host)
    got = pos.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got[:, :12], exp_pos[:, :12])
