"""GPU parity tests of the BCH path (include/ezbch.h): the HIP kernels through the C ABI against the
CPU restatement (oracle/ezbch_oracle.c) on identical seeded inputs, the reference's fixtures (README
vector, Itron SCM captures), and full-size C5 round trips (BCH(1023,983,4), 1,048,576 codewords of
122 data + 5 ECC bytes).  Bit-exact everywhere: results, corrected bytes, error locations."""
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bch_itron.npz")


@pytest.fixture(scope="module")
def torch():
    import torch as T
    if not T.cuda.is_available():
        pytest.skip("no GPU")
    return T


def _flip(rows, nbits, counts, rng):
    """Flip counts[k] distinct codeword bits (MSB first over data then ECC) of row k."""
    for k, ne in enumerate(counts):
        for p in rng.choice(nbits, int(ne), replace=False):
            rows[k, p // 8] ^= 0x80 >> (p % 8)


# (m, t): L <= 4 closed-form roots, L > 4 Chien, LDS and global field tables, unused ECC bits
CODECS = [(5, 2), (8, 2), (8, 8), (10, 4), (11, 5), (12, 5), (13, 4), (15, 4), (7, 8),
          # beyond one 64-bit remainder word and t > 8 (general BCH)
          (13, 8), (10, 9), (14, 12), (15, 16), (12, 16), (6, 10), (9, 13), (16 - 1, 9),
          # t > 16 / ECC > 256 bits: the run-time-t kernel (k_bch_decode_big), 1..16 remainder words
          (7, 17), (8, 17), (10, 20), (9, 30), (12, 30), (15, 40), (13, 64),
          # t > 64 or ECC > 1024 bits: one wavefront per codeword (k_bch_*_wave), every
          # init_bch-valid codec
          (10, 65), (12, 90), (13, 100), (15, 200), (11, 120)]
BIG = {(10, 65), (12, 90), (13, 100), (15, 200), (11, 120)}


@pytest.mark.parametrize("m,t", CODECS, ids=[f"m{m}t{t}" for m, t in CODECS])
def test_device_matches_oracle(torch, m, t):
    import ezrs
    oc, c = O.BCH(m, t), ezrs.BCH(m, t)
    assert (c.n, c.ecc_bits, c.ecc_bytes) == (oc.n, oc.ecc_bits, oc.ecc_bytes)
    rng = np.random.default_rng(1000 * m + t)
    for L in sorted({min(oc.max_len, 300), max(1, oc.max_len // 3), 1}):
        ncw = 300 if (m, t) in BIG else 2500
        eb = oc.ecc_bytes
        rows = rng.integers(0, 256, (ncw, L + eb), dtype=np.uint8)
        ref = rows.copy()
        oc.encode_batch(ref, L, nthreads=8)
        dev = torch.from_numpy(rows).cuda()
        c.encode(dev, L)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dev.cpu().numpy(), ref, err_msg=f"encode L={L}")
        # 0 .. t+2 bit errors, plus codewords whose only difference is an unused ECC bit
        bad = ref.copy()
        _flip(bad, 8 * L + oc.ecc_bits, np.arange(ncw) % (t + 3), rng)
        if 8 * eb > oc.ecc_bits:
            bad[::7, L + eb - 1] ^= 1
        exp = bad.copy()
        eloc = np.zeros((ncw, t), np.uint32)
        eres = oc.decode_batch(exp, L, errloc=eloc, nthreads=8)
        d = torch.from_numpy(bad).cuda()
        loc = torch.zeros((ncw, t), dtype=torch.int32, device="cuda")
        res = c.decode(d, L, errloc=loc).cpu().numpy()
        np.testing.assert_array_equal(res, eres, err_msg=f"result L={L}")
        np.testing.assert_array_equal(d.cpu().numpy(), exp, err_msg=f"data L={L}")
        got = loc.cpu().numpy().view(np.uint32)
        for k in np.nonzero(eres > 0)[0]:
            np.testing.assert_array_equal(got[k, :eres[k]], eloc[k, :eres[k]])
        assert (res[np.arange(ncw) % (t + 3) <= t] >= 0).all()


@pytest.mark.parametrize("L,pitch", [(95, 0), (96, 0), (97, 0), (99, 0), (101, 0), (122, 0), (127, 0),
                                     (128, 0), (129, 0), (131, 0), (200, 0), (120, 600), (130, 700)])
def test_split_remainder_lengths(torch, L, pitch):
    """1-word codecs (ecc_bits <= 64) take the four-chain remainder from 3 kQ = 96 data bytes on:
    stream 0 starting before the row (L < 128) or after a head chain (L > 128), every row
    alignment (odd strides), and rows read in place (a pitch too wide to stage in LDS)."""
    import ezrs
    oc, c = O.BCH(12, 5), ezrs.BCH(12, 5)
    eb, ncw = oc.ecc_bytes, 700
    w = max(pitch, L + eb)
    rng = np.random.default_rng(L * 31 + pitch)
    rows = rng.integers(0, 256, (ncw, w), dtype=np.uint8)
    ref = rows.copy()
    sub = ref[:, :L + eb].copy()
    oc.encode_batch(sub, L, nthreads=8)
    ref[:, :L + eb] = sub
    dev = torch.from_numpy(rows).cuda()
    c.encode(dev, L)
    np.testing.assert_array_equal(dev.cpu().numpy(), ref, err_msg="encode")
    bad = ref.copy()
    sub = bad[:, :L + eb].copy()
    _flip(sub, 8 * L + oc.ecc_bits, np.arange(ncw) % 8, rng)
    bad[:, :L + eb] = sub
    exp = bad.copy()
    eres = oc.decode_batch(sub, L, nthreads=8)
    exp[:, :L + eb] = sub
    d = torch.from_numpy(bad).cuda()
    res = c.decode(d, L).cpu().numpy()
    np.testing.assert_array_equal(res, eres, err_msg="result")
    np.testing.assert_array_equal(d.cpu().numpy(), exp, err_msg="data")


def test_separate_ecc_and_too_long(torch):
    import ezrs
    oc, c = O.BCH(10, 4), ezrs.BCH.nkt(1023, 983, 4)
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, (300, 122), dtype=np.uint8)
    ecc = np.zeros((300, 5), np.uint8)
    oc.encode_batch(data, 122, ecc)
    dd, de = torch.from_numpy(data).cuda(), torch.zeros((300, 8), dtype=torch.uint8, device="cuda")
    c.encode(dd, 122, de)
    np.testing.assert_array_equal(de.cpu().numpy()[:, :5], ecc)
    long = torch.zeros((4, 123 + 5), dtype=torch.uint8, device="cuda")
    assert (c.decode(long, 123).cpu().numpy() == -22).all()


def test_readme_and_itron_fixtures(torch):
    import ezrs
    c = ezrs.BCH.nkt(255, 239, 2)
    assert repr(c) == "BCH(255,239,2)"
    row = np.array([[0x01, 0x23, 0x45, 0x67, 0x89, 0xAB, 0xCD, 0xEF, 0, 0]], np.uint8)
    d = torch.from_numpy(row).cuda()
    c.encode(d, 8)
    assert d.cpu().numpy()[0, 8:].tolist() == [0xCB, 0xBB]       # README.org:1185-1188
    d[0, 1] ^= 1 << 3
    loc = torch.zeros((1, 2), dtype=torch.int32, device="cuda")
    assert int(c.decode(d, 8, errloc=loc).cpu()[0]) == 1
    assert int(loc.cpu()[0, 0]) == 11 and d.cpu().numpy()[0, 1] == 0x23
    with np.load(GOLD) as z:
        msg, valid = z["msg"], z["valid"]
    oc = O.BCH(8, 2)
    rows = np.ascontiguousarray(msg[:, 2:12])
    exp = rows.copy()
    eloc = np.zeros((len(rows), 2), np.uint32)
    eres = oc.decode_batch(exp, 8, errloc=eloc)
    d = torch.from_numpy(rows).cuda()
    loc = torch.zeros((len(rows), 2), dtype=torch.int32, device="cuda")
    res = c.decode(d, 8, errloc=loc).cpu().numpy()
    np.testing.assert_array_equal(res, eres)
    assert (res[valid] == 0).all()
    np.testing.assert_array_equal(d.cpu().numpy(), exp)
    got = loc.cpu().numpy().view(np.uint32)
    for k in np.nonzero(eres > 0)[0]:
        np.testing.assert_array_equal(got[k, :eres[k]], eloc[k, :eres[k]])


def test_host_forms(torch):
    import ezrs
    oc, c = O.BCH(10, 4), ezrs.BCH(10, 4)
    rng = np.random.default_rng(11)
    rows = rng.integers(0, 256, (5000, 127), dtype=np.uint8)
    ref = rows.copy()
    oc.encode_batch(ref, 122, nthreads=8)
    c.encode_host(rows, 122, chunk=1234)
    np.testing.assert_array_equal(rows, ref)
    _flip(rows, 8 * 122 + 40, np.arange(5000) % 6, rng)
    exp = rows.copy()
    eloc = np.zeros((5000, 4), np.uint32)
    eres = oc.decode_batch(exp, 122, errloc=eloc, nthreads=8)
    loc = np.zeros((5000, 4), np.uint32)
    res = c.decode_host(rows, 122, errloc=loc, chunk=999)
    np.testing.assert_array_equal(res, eres)
    np.testing.assert_array_equal(rows, exp)
    np.testing.assert_array_equal(loc, np.where(np.arange(4) < np.maximum(eres, 0)[:, None], eloc, 0))


def test_c5_full_size_round_trip(torch):
    """C5: BCH(1023,983,4), 1M codewords x (122 + 5) bytes; encode vs the oracle on a sample, then
    0..4 random bit errors per codeword must all be corrected exactly."""
    import ezrs
    c, oc = ezrs.BCH.nkt(1023, 983, 4), O.BCH(10, 4)
    ncw, L = 1 << 20, 122
    gen = torch.Generator(device="cuda").manual_seed(0x5EED0005)
    rows = torch.randint(0, 256, (ncw, L + 5), generator=gen, device="cuda", dtype=torch.int32)
    rows = rows.to(torch.uint8)
    c.encode(rows, L)
    host = rows.cpu().numpy()
    sample = host[::397].copy()
    ref = sample.copy()
    oc.encode_batch(ref, L, nthreads=8)
    np.testing.assert_array_equal(sample, ref)
    rng = np.random.default_rng(5)
    nbits = 8 * L + 40
    counts = rng.integers(0, 5, ncw)
    pos = np.sort(rng.random((ncw, 4)), axis=1)          # distinct positions per row
    pos = (pos * (nbits - 3)).astype(np.int64) + np.arange(4)   # strictly increasing, < nbits
    bad = host.copy()
    for j in range(4):
        sel = counts > j
        r, p = np.nonzero(sel)[0], pos[sel, j]
        bad[r, p // 8] ^= (0x80 >> (p % 8)).astype(np.uint8)
    d = torch.from_numpy(bad).cuda()
    res = c.decode(d, L).cpu().numpy()
    np.testing.assert_array_equal(res, counts)
    assert torch.equal(d, rows)


@pytest.mark.parametrize("m,t", [(10, 4), (13, 8), (15, 16), (13, 40), (13, 100)])
def test_decode_from_ecc_difference(torch, m, t):
    """decode_bch's recv XOR calc form (bch_base:96-111; ezbch_decode_ecc): the locations found
    from the ECC difference alone equal those of a full decode of the same corrupted codeword."""
    import ezrs
    oc, c = O.BCH(m, t), ezrs.BCH(m, t)
    rng = np.random.default_rng(7 * m + t)
    L, ncw, eb = min(oc.max_len, 200), 3000 if t <= 64 else 400, oc.ecc_bytes
    ref = rng.integers(0, 256, (ncw, L + eb), dtype=np.uint8)
    oc.encode_batch(ref, L)
    bad = ref.copy()
    _flip(bad, 8 * L + oc.ecc_bits, np.arange(ncw) % (t + 3), rng)
    exp = bad.copy()
    eloc = np.zeros((ncw, t), np.uint32)
    eres = oc.decode_batch(exp, L, errloc=eloc)
    # calc_ecc = ECC of the received data; the difference with the received ECC
    calc = bad.copy()
    oc.encode_batch(calc, L)
    diff = (calc[:, L:] ^ bad[:, L:]).copy()
    d = torch.from_numpy(diff).cuda()
    loc = torch.zeros((ncw, t), dtype=torch.int32, device="cuda")
    res = c.decode_ecc(d, L, errloc=loc).cpu().numpy()
    np.testing.assert_array_equal(res, eres)
    got = loc.cpu().numpy().view(np.uint32)
    for k in np.nonzero(eres > 0)[0]:
        np.testing.assert_array_equal(got[k, :eres[k]], eloc[k, :eres[k]])
    np.testing.assert_array_equal(d.cpu().numpy(), diff)        # nothing corrected


@pytest.mark.parametrize("m,t", [(10, 4), (13, 8), (15, 16), (10, 20), (13, 40), (12, 90)])
def test_decode_from_syndromes(torch, m, t):
    """decode_bch's syndrome form (bch_base:112-114; ezbch_decode_syn): syndromes of corrupted
    codewords give the same locations as a full decode, and arbitrary syndrome vectors (not those
    of any received word) give the oracle's result and locations."""
    import ezrs
    oc, c = O.BCH(m, t), ezrs.BCH(m, t)
    rng = np.random.default_rng(31 * m + t)
    L, eb = min(oc.max_len, 150), oc.ecc_bytes
    ncw = 1200 if t <= 64 else 300
    ref = rng.integers(0, 256, (ncw, L + eb), dtype=np.uint8)
    oc.encode_batch(ref, L)
    bad = ref.copy()
    _flip(bad, 8 * L + oc.ecc_bits, np.arange(ncw) % (t + 3), rng)
    syn = np.stack([oc.syndromes(bad[k, :L], bad[k, L:]) for k in range(ncw)])
    syn[ncw // 2:] = rng.integers(0, oc.n + 1, (ncw - ncw // 2, 2 * t))   # arbitrary vectors
    syn[-7:] = 0                                                           # all-zero syndromes
    exp = [oc.decode_syn(L, syn[k]) for k in range(ncw)]
    d = torch.from_numpy(syn.view(np.int32)).cuda()
    loc = torch.zeros((ncw, t), dtype=torch.int32, device="cuda")
    res = c.decode_syn(d, L, errloc=loc).cpu().numpy()
    np.testing.assert_array_equal(res, [r for r, _ in exp])
    got = loc.cpu().numpy().view(np.uint32)
    for k in range(ncw):
        if exp[k][0] > 0:
            np.testing.assert_array_equal(got[k, :exp[k][0]], exp[k][1])
    full = bad[:ncw // 2].copy()
    assert (res[:ncw // 2] == oc.decode_batch(full, L)).all()


def test_decode_syn_host_form(torch):
    """ezbch_decode_syn_host (the classic decode_bch(..., syn, errloc) behind include/ezpwd/bch):
    host syndrome rows in, results and locations out, equal to the oracle."""
    import ctypes as C
    import ezrs
    m, t, L = 10, 4, 100
    oc, c = O.BCH(m, t), ezrs.BCH(m, t)
    rng = np.random.default_rng(5)
    ncw = 64
    ref = rng.integers(0, 256, (ncw, L + oc.ecc_bytes), dtype=np.uint8)
    oc.encode_batch(ref, L)
    _flip(ref, 8 * L + oc.ecc_bits, np.arange(ncw) % (t + 3), rng)
    syn = np.ascontiguousarray(np.stack([oc.syndromes(ref[k, :L], ref[k, L:]) for k in range(ncw)]))
    res = np.zeros(ncw, np.int32)
    loc = np.zeros((ncw, t), np.uint32)
    L_ = ezrs.lib()
    L_.ezbch_decode_syn_host.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint, C.c_void_p,
                                         C.c_void_p, C.c_size_t, C.c_size_t]
    assert L_.ezbch_decode_syn_host(c._h, syn.ctypes.data, 2 * t, L, res.ctypes.data, loc.ctypes.data,
                                    t, ncw) == 0
    for k in range(ncw):
        er, el = oc.decode_syn(L, syn[k])
        assert res[k] == er
        if er > 0:
            np.testing.assert_array_equal(loc[k, :er], el)


def test_c5_packed_rows_at_odd_offset(torch):
    """the C5 decode's write-back of corrected 16-byte pieces when the rows' base is not
    16-byte aligned (a view at byte offset 3 of packed 127-byte rows): the row base's misalignment
    and the edge pieces written byte by byte.  Errors in the first and last rows of every 64-row
    wave and in random others; bytes outside the rows must stay untouched."""
    import ezrs
    oc, c = O.BCH(10, 4), ezrs.BCH.nkt(1023, 983, 4)
    L, eb = 122, 5
    ncw = 5000
    rng = np.random.default_rng(0xB5)
    rows = rng.integers(0, 256, (ncw, L + eb), dtype=np.uint8)
    oc.encode_batch(rows, L, nthreads=8)
    bad = rows.copy()
    counts = np.zeros(ncw, np.int64)
    k = np.arange(ncw)
    counts[(k % 64 == 0) | (k % 64 == 63)] = 4
    counts[rng.choice(ncw, 800, replace=False)] = rng.integers(1, 5, 800)
    _flip(bad, 8 * L + oc.ecc_bits, counts, rng)
    exp = bad.copy()
    eres = oc.decode_batch(exp, L, nthreads=8)
    for off in (3, 9):
        flat = torch.from_numpy(rng.integers(0, 256, ncw * (L + eb) + 32, dtype=np.uint8)).cuda()
        guard = flat.clone()
        view = flat[off:off + ncw * (L + eb)].view(ncw, L + eb)
        view.copy_(torch.from_numpy(bad).cuda())
        res = c.decode(view, L).cpu().numpy()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(res, eres, err_msg=f"result off={off}")
        np.testing.assert_array_equal(view.cpu().numpy(), exp, err_msg=f"rows off={off}")
        f = flat.cpu().numpy()
        g = guard.cpu().numpy()
        np.testing.assert_array_equal(f[:off], g[:off])
        np.testing.assert_array_equal(f[off + ncw * (L + eb):], g[off + ncw * (L + eb):])


@pytest.mark.parametrize("ncw", [1, 2, 5, 255, 256, 257, 767])
def test_c5_plane_sliced_small_batches(torch, ncw):
    """The plane-sliced encode and fused decode (ezbch_ps_tile.hpp) on batches of one partial tile,
    exactly one, and a few: the first tile's guard bytes, the span-end re-read of the last row, rows
    past the batch dropped by the buffer range checks.  Encode into packed rows (ECC inline) and
    into a separate ECC array, then decode 0..4 (and 5, uncorrectable) bit errors per row against
    the oracle, with error locations."""
    import ezrs
    oc, c = O.BCH(10, 4), ezrs.BCH.nkt(1023, 983, 4)
    L, eb = 122, 5
    rng = np.random.default_rng(0xC5 + ncw)
    rows = rng.integers(0, 256, (ncw, L + eb), dtype=np.uint8)
    ref = rows.copy()
    oc.encode_batch(ref, L, nthreads=8)
    dev = torch.from_numpy(rows).cuda()
    c.encode(dev, L)                                      # ECC inline
    np.testing.assert_array_equal(dev.cpu().numpy(), ref)
    data = torch.from_numpy(np.ascontiguousarray(rows[:, :L])).cuda()
    ecc = torch.zeros((ncw, eb), dtype=torch.uint8, device="cuda")
    c.encode(data, L, ecc=ecc)                            # separate ECC array
    np.testing.assert_array_equal(ecc.cpu().numpy(), ref[:, L:])
    bad = ref.copy()
    _flip(bad, 8 * L + oc.ecc_bits, np.arange(ncw) % 6, rng)
    exp = bad.copy()
    eloc = np.zeros((ncw, 4), np.uint32)
    eres = oc.decode_batch(exp, L, errloc=eloc, nthreads=8)
    d = torch.from_numpy(bad).cuda()
    loc = torch.zeros((ncw, 4), dtype=torch.int32, device="cuda")
    res = c.decode(d, L, errloc=loc).cpu().numpy()
    np.testing.assert_array_equal(res, eres)
    np.testing.assert_array_equal(d.cpu().numpy(), exp)
    got = loc.cpu().numpy().view(np.uint32)
    for k in np.nonzero(eres > 0)[0]:
        np.testing.assert_array_equal(got[k, :eres[k]], eloc[k, :eres[k]])
