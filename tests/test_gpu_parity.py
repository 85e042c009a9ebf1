"""GPU parity tests: the HIP engine through the C ABI against the reference's golden vectors and
the oracle (CPU restatement) on identical seeded inputs.  Bit-exact equality everywhere."""
import numpy as np
import pytest

import oracle as O
from golden_util import fixture_files, fixture_id, load

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as T
    if not T.cuda.is_available():
        pytest.skip("no GPU")
    return T


def _codec(params):
    import ezrs
    mm, poly, fcr, prim, nroots, dual = (int(x) for x in params)
    return ezrs.Codec(mm, poly, fcr, prim, nroots, bool(dual))


def _tdt(torch, dt):
    return torch.uint8 if dt == np.uint8 else torch.uint16


def _to_dev(torch, a):
    if a.dtype == np.uint16:
        return torch.from_numpy(a.view(np.int16)).view(torch.uint16).cuda()
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _to_np(t, dt):
    t = t.cpu()
    if dt == np.uint16:
        return t.view(__import__("torch").int16).numpy().view(np.uint16)
    return t.numpy()


@pytest.mark.parametrize("fn", fixture_files(), ids=fixture_id)
def test_golden_device(torch, fn):
    f = load(fn)
    c = _codec(f["params"])
    dt = c.dtype
    nr = c.nroots
    for t in range(len(f["length"])):
        L = int(f["length"][t])
        d = _to_dev(torch, f["enc_data"][t:t + 1, :L].copy())
        p = torch.zeros((1, nr), dtype=_tdt(torch, dt), device="cuda")
        c.encode(d, L, p)
        np.testing.assert_array_equal(_to_np(p, dt)[0], f["enc_parity"][t], err_msg=f"enc t={t}")

        d = _to_dev(torch, f["dec_data_in"][t:t + 1, :L].copy())
        p = _to_dev(torch, f["dec_parity_in"][t:t + 1].copy())
        corr = _to_dev(torch, f["dec_corr_in"][t:t + 1].copy())
        ne = int(f["dec_neras"][t])
        eras = torch.from_numpy(f["dec_eras"][t:t + 1].astype(np.int32)).cuda()
        neras = torch.tensor([ne], dtype=torch.int32, device="cuda")
        pos = torch.zeros((1, max(nr, 1)), dtype=torch.int32, device="cuda")
        r = c.decode(d, L, p, eras=eras, neras=neras, positions=pos, corr=corr)
        torch.cuda.synchronize()
        res = int(r.cpu()[0])
        assert res == f["dec_result"][t], f"t={t}"
        np.testing.assert_array_equal(pos.cpu().numpy()[0, :max(res, 0)].astype(np.uint32),
                                      f["dec_positions"][t, :max(res, 0)])
        np.testing.assert_array_equal(_to_np(d, dt)[0], f["dec_data_out"][t, :L])
        np.testing.assert_array_equal(_to_np(p, dt)[0], f["dec_parity_out"][t])
        np.testing.assert_array_equal(_to_np(corr, dt)[0], f["dec_corr_out"][t])


@pytest.mark.parametrize("fn", fixture_files()[::3], ids=fixture_id)
def test_golden_host_pipeline(torch, fn):
    f = load(fn)
    c = _codec(f["params"])
    nr = c.nroots
    for t in range(len(f["length"])):
        L = int(f["length"][t])
        d = f["enc_data"][t:t + 1, :L].copy()
        p = np.zeros((1, nr), c.dtype)
        c.encode_host(d, L, p)
        np.testing.assert_array_equal(p[0], f["enc_parity"][t])
        d = f["dec_data_in"][t:t + 1, :L].copy()
        p = f["dec_parity_in"][t:t + 1].copy()
        ne = int(f["dec_neras"][t])
        eras = f["dec_eras"][t:t + 1].copy()
        neras = np.array([ne], np.uint32)
        pos = np.zeros((1, nr), np.uint32)
        r = c.decode_host(d, L, p, eras=eras, neras=neras, positions=pos)
        assert r[0] == f["dec_result"][t]
        np.testing.assert_array_equal(pos[0, :max(r[0], 0)], f["dec_positions"][t, :max(r[0], 0)])
        np.testing.assert_array_equal(d[0], f["dec_data_out"][t, :L])
        np.testing.assert_array_equal(p[0], f["dec_parity_out"][t])


@pytest.mark.parametrize("n,k,pad,pinned", [(255, 223, 0, False), (255, 223, 5, True),
                                              (255, 251, 3, False), (1023, 991, 0, True)])
def test_host_pipeline_inline_parity(torch, n, k, pad, pinned):
    """Host forms with parity inside the row (the linear-copy path), several chunks, pageable and
    pinned buffers: encode, then an 8-error/4-erasure (t=2 codecs: 1+1) decode, against the oracle."""
    import ezrs
    c = ezrs.Codec.rs(n, k)
    oc = O.Codec(*O.rs_params(n, k))
    nr = n - k
    rng = np.random.default_rng(n * 7 + k + pad)
    ncw, stride = 2500, n + pad
    host = rng.integers(0, n + 1, (ncw, stride)).astype(c.dtype)
    exp = host.copy()
    oc.encode_batch(exp, k)
    buf = torch.from_numpy(host.view(np.int16) if c.dtype == np.uint16 else host)
    if pinned:
        buf = buf.pin_memory()
    h = buf.numpy().view(c.dtype)
    c.encode_host(h, k, chunk=700)
    np.testing.assert_array_equal(h, exp)                     # parity written, pad untouched
    ne, nx = (8, 4) if nr >= 16 else (1, 1)
    locs = np.argsort(rng.random((ncw, n)), axis=1)[:, :ne + nx]
    rows = np.arange(ncw)[:, None]
    h[rows, locs] ^= rng.integers(1, n + 1, (ncw, ne + nx)).astype(c.dtype)
    eras = np.zeros((ncw, nr), np.uint32)
    eras[:, :nx] = locs[:, ne:]
    neras = np.full(ncw, nx, np.uint32)
    r = c.decode_host(h, k, eras=eras, neras=neras, chunk=700)
    assert (r == ne + nx).all()
    np.testing.assert_array_equal(h, exp)


@pytest.mark.parametrize("pinned", [False, True])
def test_host_pipeline_sparse_changes(torch, pinned):
    """decode_host brings back only the rows whose result is nonzero (compacted on the device):
    5% of the rows correctable, 1% overwhelmed (partial corrections kept, rs_base:1238-1241), the
    rest clean, over several chunks and both pipeline streams -- every row and result equals the
    oracle's."""
    import ezrs
    c = ezrs.Codec.rs(255, 223)
    oc = O.Codec(*O.rs_params(255, 223))
    rng = np.random.default_rng(77)
    ncw, stride = 9000, 258
    host = rng.integers(0, 256, (ncw, stride)).astype(np.uint8)
    oc.encode_batch(host, 223)
    pick = rng.random(ncw)
    for kk in np.nonzero(pick < 0.06)[0]:
        m = 40 if pick[kk] < 0.01 else int(rng.integers(1, 17))
        locs = rng.choice(255, m, replace=False)
        host[kk, locs] ^= rng.integers(1, 256, m).astype(np.uint8)
    exp = host.copy()
    exp_r = oc.decode_batch(exp, 223)
    buf = torch.from_numpy(host)
    if pinned:
        buf = buf.pin_memory()
    h = buf.numpy()
    r = c.decode_host(h, 223, chunk=1000)
    np.testing.assert_array_equal(r, exp_r)
    np.testing.assert_array_equal(h, exp)
    assert (r == -1).any() and (r > 0).any() and (r == 0).mean() > 0.9


@pytest.mark.parametrize("n,k,ncw,L", [(65535, 65503, 6, 65503), (65535, 65503, 40, 900),
                                        (1023, 1001, 300, 1001), (4095, 4063, 50, 2000)])
def test_wide_symbol_lane_kernels_vs_oracle(torch, n, k, ncw, L):
    """m > 8, NR <= 32: the lane-group encode and syndrome/decode kernels against the oracle --
    parity, result, positions and corrected rows -- with 8 errors + 4 erasures per row."""
    import ezrs
    c = ezrs.Codec.rs(n, k)
    oc = O.Codec(*O.rs_params(n, k))
    nr = n - k
    rng = np.random.default_rng(n + ncw)
    host = rng.integers(0, n + 1, (ncw, L + nr)).astype(np.uint16)
    ref = host.copy()
    oc.encode_batch(ref, L)
    dev = _to_dev(torch, host)
    c.encode(dev, L)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_to_np(dev, np.uint16), ref)
    bad = ref.copy()
    locs = np.stack([rng.choice(L + nr, 12, replace=False) for _ in range(ncw)])
    rows = np.arange(ncw)[:, None]
    bad[rows, locs] ^= rng.integers(1, n + 1, (ncw, 12)).astype(np.uint16)
    eras = np.zeros((ncw, nr), np.uint32)
    eras[:, :4] = locs[:, 8:]
    neras = np.full(ncw, 4, np.uint32)
    exp = bad.copy()
    exp_pos = np.zeros((ncw, nr), np.uint32)
    exp_r = oc.decode_batch(exp, L, None, eras, neras, exp_pos)
    d = _to_dev(torch, bad)
    pos = torch.zeros((ncw, nr), dtype=torch.int32, device="cuda")
    r = c.decode(d, L, eras=torch.from_numpy(eras.view(np.int32)).cuda(),
                 neras=torch.from_numpy(neras.view(np.int32)).cuda(), positions=pos)
    torch.cuda.synchronize()
    r = r.cpu().numpy()
    np.testing.assert_array_equal(r, exp_r)
    np.testing.assert_array_equal(_to_np(d, np.uint16), exp)
    got_pos = pos.cpu().numpy().view(np.uint32)
    for i in range(ncw):
        if r[i] > 0:
            np.testing.assert_array_equal(got_pos[i, :r[i]], exp_pos[i, :r[i]])


def _inject(torch, cw, n_err, n_era, nn, gen):
    """Corrupt n_err + n_era distinct symbols per row; the last n_era are flagged as erasures."""
    ncw, n = cw.shape
    keys = torch.rand((ncw, n), generator=gen, device=cw.device)
    locs = keys.argsort(dim=1)[:, :n_err + n_era]
    vals = torch.randint(1, nn + 1, (ncw, n_err + n_era), generator=gen, device=cw.device,
                         dtype=torch.int32).to(cw.dtype)
    cw.scatter_(1, locs, cw.gather(1, locs) ^ vals)
    eras = locs[:, n_err:].to(torch.int32).contiguous()
    return locs, eras


# the 17 codecs rsvalidate cross-checks against Karn (rsvalidate.C:46-62), plus CCSDS; every
# RS(255,K) with NROOTS <= 32 and RS_CCSDS_CONV(255,239) run the plane-sliced tile kernels
RSVALIDATE_NR = [1, 2, 3, 4, 7, 9, 12, 16, 17, 27, 46, 77, 99, 127, 128, 129, 199]
BULK = ([("RS(255,223)", 1 << 16), ("RS_CCSDS(255,223)", 1 << 16), ("RS(255,251)", 1 << 16),
         ("RS_CCSDS_CONV(255,239)", 1 << 14)] +
        [(f"RS(255,{255 - nr})", 1 << 12) for nr in RSVALIDATE_NR if nr not in (4, 32)])


@pytest.mark.parametrize("maker,ncw", BULK)
def test_bulk_vs_oracle(torch, maker, ncw):
    """Random shortened length, error loads 0..3x capacity: every output equals the oracle's
    (result, positions, corrected data and parity); 64k codewords for the headline codecs, 4k for
    the rest of rsvalidate's set.  Codecs with NROOTS <= 32 must be on the plane-sliced path."""
    import ezrs
    if maker.startswith("RS("):
        c = ezrs.Codec.rs(255, int(maker[7:-1]))
        oc = O.Codec(*O.rs_params(255, c.load))
    elif maker.startswith("RS_CCSDS_CONV"):
        c = ezrs.Codec.ccsds(239, dual=False)
        oc = O.Codec(*O.ccsds_params(239, False))
    else:
        c = ezrs.Codec.ccsds(223)
        oc = O.Codec(*O.ccsds_params(223))
    if c.nroots <= 32 and not c.dual:
        assert c.kernel_path == "planeslice", (maker, c.kernel_path)
    rng = np.random.default_rng(11)
    L, nr = c.load - 17, c.nroots
    data = rng.integers(0, 256, (ncw, L + nr)).astype(np.uint8)
    ref = data.copy()
    oc.encode_batch(ref, L, None, nthreads=8)
    dev = torch.from_numpy(data).cuda()
    c.encode(dev, L)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dev.cpu().numpy(), ref)
    # corrupt the oracle's codewords with varying loads
    load = rng.integers(0, min(3 * nr // 2, L + nr) + 1, ncw)
    cw = ref.copy()
    eras = np.zeros((ncw, nr), np.uint32)
    neras = np.zeros(ncw, np.uint32)
    for k in range(ncw):
        m = int(load[k])
        locs = rng.choice(L + nr, m, replace=False)
        cw[k, locs] ^= rng.integers(1, 256, m).astype(np.uint8)
        ne = min(int(rng.integers(0, m + 1)), nr)
        eras[k, :ne] = locs[:ne]
        neras[k] = ne
    exp = cw.copy()
    exp_pos = np.zeros((ncw, nr), np.uint32)
    exp_r = oc.decode_batch(exp, L, None, eras, neras, exp_pos, nthreads=8)
    dcw = torch.from_numpy(cw).cuda()
    pos = torch.zeros((ncw, nr), dtype=torch.int32, device="cuda")
    r = c.decode(dcw, L, None, eras=torch.from_numpy(eras.view(np.int32)).cuda(),
                 neras=torch.from_numpy(neras.view(np.int32)).cuda(), positions=pos)
    torch.cuda.synchronize()
    r = r.cpu().numpy()
    np.testing.assert_array_equal(r, exp_r)
    np.testing.assert_array_equal(dcw.cpu().numpy(), exp)
    pos = pos.cpu().numpy().view(np.uint32)
    for k in np.nonzero(r > 0)[0]:
        np.testing.assert_array_equal(pos[k, :r[k]], exp_pos[k, :r[k]])
    assert (r == -1).any() and (r == 0).any() and (r > 0).any()


def test_c2_c3_full_size(torch):
    """BASELINE configs C2/C3 at full size (1M RS(255,223) codewords): encode parity equals the
    oracle on a sample; clean decode returns 0 everywhere; 8 errors + 4 erasures per codeword
    decode to result 12 with the original codewords restored (size-independent properties)."""
    import ezrs
    c = ezrs.Codec.rs(255, 223)
    oc = O.Codec(*O.rs_params(255, 223))
    ncw = 1 << 20
    gen = torch.Generator(device="cuda").manual_seed(0x5EED0002)
    cw = torch.randint(0, 256, (ncw, 255), generator=gen, device="cuda", dtype=torch.int32)
    cw = cw.to(torch.uint8)
    c.encode(cw, 223)
    torch.cuda.synchronize()
    host = cw.cpu().numpy()
    sample = host[::61].copy()
    exp = sample.copy()
    oc.encode_batch(exp, 223, None, nthreads=8)
    np.testing.assert_array_equal(sample, exp)
    clean = cw.clone()
    r = c.decode(clean, 223)
    torch.cuda.synchronize()
    assert int((r != 0).sum()) == 0
    assert torch.equal(clean, cw)
    bad = cw.clone()
    locs, eras = _inject(torch, bad, 8, 4, 255, gen)
    neras = torch.full((ncw,), 4, dtype=torch.int32, device="cuda")
    pos = torch.zeros((ncw, 32), dtype=torch.int32, device="cuda")
    r = c.decode(bad, 223, eras=eras, neras=neras, positions=pos)
    torch.cuda.synchronize()
    assert int((r != 12).sum()) == 0
    assert torch.equal(bad, cw)
    exp_pos = locs.sort(dim=1).values.to(torch.int32)       # PRIM = 1: ascending order
    assert torch.equal(pos[:, :12], exp_pos)


def test_c2_past_infinity_cache(torch):
    """4M RS(255,223) codewords (1.07 GB, past the 256 MiB Infinity Cache): parity equals the oracle
    on rows sampled across the whole batch (every tile and launch chunk boundary region), clean
    decode returns 0 everywhere, and 8 errors per codeword spread over the batch decode back to
    the original rows."""
    import ezrs
    c = ezrs.Codec.rs(255, 223)
    oc = O.Codec(*O.rs_params(255, 223))
    ncw = 4 << 20
    gen = torch.Generator(device="cuda").manual_seed(0x5EED0004)
    cw = torch.randint(0, 256, (ncw, 255), generator=gen, device="cuda", dtype=torch.int32)
    cw = cw.to(torch.uint8)
    c.encode(cw, 223)
    torch.cuda.synchronize()
    idx = np.unique(np.concatenate([np.arange(0, ncw, 997), np.arange(ncw - 300, ncw),
                                    np.arange(0, 300)]))
    sample = cw[torch.from_numpy(idx).cuda()].cpu().numpy()
    exp = sample.copy()
    oc.encode_batch(exp, 223, None, nthreads=8)
    np.testing.assert_array_equal(sample, exp)
    clean = cw.clone()
    r = c.decode(clean, 223)
    torch.cuda.synchronize()
    assert int((r != 0).sum()) == 0 and torch.equal(clean, cw)
    bad = cw.clone()
    _inject(torch, bad, 8, 0, 255, gen)
    r = c.decode(bad, 223)
    torch.cuda.synchronize()
    assert int((r != 8).sum()) == 0
    assert torch.equal(bad, cw)


@pytest.mark.parametrize("maker", ["RS(255,223)", "RS_CCSDS(255,223)", "RS_CCSDS_CONV(255,223)",
                                   "RS(255,239)", "RS(255,251)"])
@pytest.mark.parametrize("L,ncw,extra", [(1, 1, 0), (2, 511, 3), (63, 513, 0), (64, 777, 5),
                                         (100, 1025, 1), (191, 600, 0)])
def test_shapes_vs_oracle(torch, maker, L, ncw, extra):
    """Shortened lengths (front padding of every width), batch sizes around the 512-codeword tile,
    row strides wider than the codeword, and a separate parity buffer for encode."""
    import ezrs
    if maker.startswith("RS_CCSDS_CONV"):
        c, params = ezrs.Codec.ccsds(223, dual=False), O.ccsds_params(223, False)
    elif maker.startswith("RS_CCSDS"):
        c, params = ezrs.Codec.ccsds(223), O.ccsds_params(223)
    else:
        k = int(maker[7:-1])
        c, params = ezrs.Codec.rs(255, k), O.rs_params(255, k)
    oc = O.Codec(*params)
    nr = c.nroots
    L = min(L, c.load)
    rng = np.random.default_rng(L * 1000 + ncw)
    stride = L + nr + extra
    data = rng.integers(0, 256, (ncw, stride)).astype(np.uint8)
    # encode into a separate parity buffer
    par = np.zeros((ncw, nr), np.uint8)
    exp_par = np.zeros((ncw, nr), np.uint8)
    oc.encode_batch(data, L, exp_par, nthreads=8)
    dd = torch.from_numpy(data).cuda()
    dp = torch.from_numpy(par).cuda()
    c.encode(dd, L, dp)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dp.cpu().numpy(), exp_par)
    # decode contiguous codewords (parity in-row), a few corrupted
    cw = data.copy()
    cw[:, L:L + nr] = exp_par
    for k in range(0, ncw, 3):
        m = int(rng.integers(1, nr // 2 + 2))
        locs = rng.choice(L + nr, min(m, L + nr), replace=False)
        cw[k, locs] ^= rng.integers(1, 256, len(locs)).astype(np.uint8)
    exp = cw.copy()
    exp_pos = np.zeros((ncw, nr), np.uint32)
    exp_r = oc.decode_batch(exp, L, None, positions=exp_pos, nthreads=8)
    dcw = torch.from_numpy(cw).cuda()
    pos = torch.zeros((ncw, nr), dtype=torch.int32, device="cuda")
    r = c.decode(dcw, L, None, positions=pos)
    torch.cuda.synchronize()
    r = r.cpu().numpy()
    np.testing.assert_array_equal(r, exp_r)
    np.testing.assert_array_equal(dcw.cpu().numpy(), exp)
    pos = pos.cpu().numpy().view(np.uint32)
    for k in np.nonzero(r > 0)[0]:
        np.testing.assert_array_equal(pos[k, :r[k]], exp_pos[k, :r[k]])


@pytest.mark.parametrize("maker", ["RS(255,223)", "RS_CCSDS_CONV(255,239)", "RS(255,247)"])
def test_erasure_split_vs_oracle(torch, maker):
    """1..4 erasures (the error path's Chien over lambda / Gamma): erasures on corrupted and on
    clean positions, repeated erasure positions, and error loads past capacity, against the
    oracle's result, positions and corrected rows."""
    import ezrs
    if maker.startswith("RS_CCSDS_CONV"):
        c, oc = ezrs.Codec.ccsds(239, dual=False), O.Codec(*O.ccsds_params(239, False))
    else:
        k = int(maker[7:-1])
        c, oc = ezrs.Codec.rs(255, k), O.Codec(*O.rs_params(255, k))
    assert c.kernel_path == "planeslice"
    rng = np.random.default_rng(23)
    ncw, nr = 20000, c.nroots
    L = c.load - int(rng.integers(0, 40))
    ref = rng.integers(0, 256, (ncw, L + nr)).astype(np.uint8)
    oc.encode_batch(ref, L, None, nthreads=8)
    cw = ref.copy()
    eras = np.zeros((ncw, nr), np.uint32)
    neras = np.zeros(ncw, np.uint32)
    for k in range(ncw):
        ne = int(rng.integers(1, 5)) if nr >= 4 else int(rng.integers(1, nr + 1))
        nerr = int(rng.integers(0, (nr - ne) // 2 + 3))          # up to 2 past capacity
        locs = rng.choice(L + nr, nerr + ne, replace=False)
        cw[k, locs[:nerr]] ^= rng.integers(1, 256, nerr).astype(np.uint8)
        kind = k % 4
        if kind == 0:
            e = locs[nerr:]                                         # clean positions
        elif kind == 1:
            e = locs[:ne] if nerr >= ne else locs[nerr:]            # on corrupted positions
        elif kind == 2:
            e = np.concatenate([locs[nerr:], locs[:0]])
            if ne >= 2:
                e = e.copy(); e[-1] = e[0]                          # a repeated position
        else:
            e = locs[nerr:].copy()
            cw[k, e[0]] ^= 0x3C                                      # an erased symbol also wrong
        eras[k, :ne] = e[:ne]
        neras[k] = ne
    exp = cw.copy()
    exp_pos = np.zeros((ncw, nr), np.uint32)
    exp_r = oc.decode_batch(exp, L, None, eras, neras, exp_pos, nthreads=8)
    dcw = torch.from_numpy(cw).cuda()
    pos = torch.zeros((ncw, nr), dtype=torch.int32, device="cuda")
    r = c.decode(dcw, L, None, eras=torch.from_numpy(eras.view(np.int32)).cuda(),
                 neras=torch.from_numpy(neras.view(np.int32)).cuda(), positions=pos)
    r = r.cpu().numpy()
    np.testing.assert_array_equal(r, exp_r)
    np.testing.assert_array_equal(dcw.cpu().numpy(), exp)
    pos = pos.cpu().numpy().view(np.uint32)
    for k in np.nonzero(r > 0)[0]:
        np.testing.assert_array_equal(pos[k, :r[k]], exp_pos[k, :r[k]])
    assert (r == -1).any() and (r > 0).any()
