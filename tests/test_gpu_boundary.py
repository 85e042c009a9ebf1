"""GPU tests of the drop-in boundary contract (include/ezrs.h):

* one const codec shared by two streams: an encode on stream A and a decode on stream B, issued
  back to back without synchronisation, each with its own per-stream workspace -- both bit-exact
  against the oracle (the reference's codec is const and shareable, rs_base:602-605);
* the caller-owned workspace forms (ezrs_encode_ws / ezrs_decode_ws) give the same results;
* ezrs_encode_host never writes the caller's data (a read-only numpy array works), brings back
  only the parity, and handles padded rows (pitch far above the row) through the gather path."""
import ctypes as C

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


def _batch(rng, ncw, n=255):
    return rng.integers(0, 256, (ncw, n)).astype(np.uint8)


def test_two_streams_share_one_codec(torch):
    import ezrs
    c = ezrs.Codec.rs(255, 223)
    oc = O.Codec(*O.rs_params(255, 223))
    rng = np.random.default_rng(0xB0B)
    ncw = 200_000
    a = _batch(rng, ncw)
    b = a.copy()
    oc.encode_batch(b, 223)                      # b: valid codewords
    bad = b.copy()
    locs = np.argsort(rng.random((ncw, 255)), axis=1)[:, :10]
    bad[np.arange(ncw)[:, None], locs] ^= rng.integers(1, 256, (ncw, 10)).astype(np.uint8)
    exp_a = a.copy()
    oc.encode_batch(exp_a, 223)
    exp_r = oc.decode_batch(bad.copy(), 223)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    da = torch.from_numpy(a).cuda()
    db = torch.from_numpy(bad).cuda()
    rbs = [torch.empty(ncw, dtype=torch.int32, device="cuda") for _ in range(3)]
    torch.cuda.synchronize()
    for rb in rbs:                               # repeated, interleaved, unsynchronised issue
        c.encode(da, 223, stream=sa)
        c.decode(db, 223, result=rb, stream=sb)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(da.cpu().numpy(), exp_a)
    # the first decode corrects 10 symbols per codeword (exp_r, the oracle's result); the two
    # repeats then see clean codewords and report 0
    assert (exp_r == 10).all()
    np.testing.assert_array_equal(rbs[0].cpu().numpy(), exp_r)
    assert (rbs[1].cpu().numpy() == 0).all() and (rbs[2].cpu().numpy() == 0).all()
    np.testing.assert_array_equal(db.cpu().numpy(), b)


def test_caller_workspace_forms(torch):
    import ezrs
    L = ezrs.lib()
    c = ezrs.Codec.rs(255, 239)
    oc = O.Codec(*O.rs_params(255, 239))
    rng = np.random.default_rng(7)
    ncw = 5000
    h = _batch(rng, ncw)
    exp = h.copy()
    oc.encode_batch(exp, 239)
    d = torch.from_numpy(h).cuda()
    par = torch.empty((ncw, 16), dtype=torch.uint8, device="cuda")
    nb = c.workspace_bytes(ncw)
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    assert L.ezrs_encode_ws(c._h, C.c_void_p(d.data_ptr()), 255, 239, C.c_void_p(par.data_ptr()),
                            16, ncw, C.c_void_p(ws.data_ptr()), nb, C.c_void_p(s)) == 0
    # a workspace one byte short is refused (no silent overrun)
    if nb:
        assert L.ezrs_encode_ws(c._h, C.c_void_p(d.data_ptr()), 255, 239,
                                C.c_void_p(par.data_ptr()), 16, ncw, C.c_void_p(ws.data_ptr()),
                                nb - 1, C.c_void_p(s)) < 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(par.cpu().numpy(), exp[:, 239:])
    d[:, 239:] = par
    res = torch.empty(ncw, dtype=torch.int32, device="cuda")
    assert L.ezrs_decode_ws(c._h, C.c_void_p(d.data_ptr()), 255, 239, None, 0, None, 0, None,
                            C.c_void_p(res.data_ptr()), None, 0, None, 0, ncw,
                            C.c_void_p(ws.data_ptr()), nb, C.c_void_p(s)) == 0
    torch.cuda.synchronize()
    assert (res.cpu().numpy() == 0).all()


@pytest.mark.parametrize("pitch", [255, 300, 4096])
def test_encode_host_reads_only(torch, pitch):
    """Rows of `pitch` bytes (255: packed; 4096: padded records -> gather path) with a separate
    parity array; the data array is read-only, so any write to it would fault."""
    import ezrs
    c = ezrs.Codec.rs(255, 223)
    oc = O.Codec(*O.rs_params(255, 223))
    rng = np.random.default_rng(pitch)
    ncw = 3000
    rows = rng.integers(0, 256, (ncw, pitch)).astype(np.uint8)
    before = rows.copy()
    rows.flags.writeable = False
    par = np.zeros((ncw, 32), np.uint8)
    c.encode_host(rows, 223, par, chunk=1000)
    np.testing.assert_array_equal(rows, before)
    exp = before[:, :255].copy()
    oc.encode_batch(exp, 223)
    badrows = np.nonzero((par != exp[:, 223:]).any(axis=1))[0]
    assert len(badrows) == 0, (badrows[:16], [np.nonzero(par[r] != exp[r, 223:])[0] for r in badrows[:4]])
    # parity scattered into a strided array (row pitch 40) lands in place, the rest untouched
    par2 = np.full((ncw, 40), 0xEE, np.uint8)
    c.encode_host(rows, 223, par2, chunk=777)
    np.testing.assert_array_equal(par2[:, :32], exp[:, 223:])
    assert (par2[:, 32:] == 0xEE).all()


def test_encode_rows_host_writes_parity_only(torch):
    import ezrs
    c = ezrs.Codec.rs(255, 223)
    oc = O.Codec(*O.rs_params(255, 223))
    rng = np.random.default_rng(11)
    ncw, pitch = 2000, 260
    rows = rng.integers(0, 256, (ncw, pitch)).astype(np.uint8)
    exp = rows.copy()
    e2 = rows[:, :255].copy()
    oc.encode_batch(e2, 223)
    exp[:, :255] = e2
    c.encode_host(rows, 223, chunk=600)        # parity None: the row form
    np.testing.assert_array_equal(rows, exp)    # data and the 5 pad bytes unchanged


def test_decode_host_single_codeword_zero_eras_stride(torch):
    """One codeword, eras_stride 0: the erasure list is taken from neras[0]."""
    import ezrs
    L = ezrs.lib()
    c = ezrs.Codec.rs(255, 223)
    oc = O.Codec(*O.rs_params(255, 223))
    rng = np.random.default_rng(3)
    row = rng.integers(0, 256, (1, 255)).astype(np.uint8)
    oc.encode_batch(row, 223)
    good = row.copy()
    row[0, [5, 77, 200]] ^= 0x5A
    eras = np.array([77, 200], np.uint32)
    neras = np.array([2], np.uint32)
    res = np.zeros(1, np.int32)
    pos = np.zeros(32, np.uint32)
    rc = L.ezrs_decode_host(c._h, row.ctypes.data_as(C.c_void_p), 255, 223, None, 0,
                            eras.ctypes.data_as(C.c_void_p), 0, neras.ctypes.data_as(C.c_void_p),
                            res.ctypes.data_as(C.c_void_p), pos.ctypes.data_as(C.c_void_p), 32,
                            None, 0, 1, 0)
    assert rc == 0 and res[0] == 3
    np.testing.assert_array_equal(row, good)
    assert sorted(pos[:3].tolist()) == [5, 77, 200]


def test_decode_null_eras_with_stride(torch):
    """eras = NULL with a nonzero eras_stride: the error path must not read erasures
    (the 16-byte erasure preload is gated on a non-null list), and a corrupted codeword among clean
    ones is still corrected exactly as the oracle does."""
    import ezrs
    L = ezrs.lib()
    c = ezrs.Codec.rs(255, 223)
    oc = O.Codec(*O.rs_params(255, 223))
    rng = np.random.default_rng(0xE5)
    ncw = 300
    h = _batch(rng, ncw)
    oc.encode_batch(h, 223)
    good = h.copy()
    h[17, [3, 99, 250]] ^= np.array([0x11, 0x22, 0x33], np.uint8)
    exp = oc.decode_batch(h.copy(), 223)
    d = torch.from_numpy(h).cuda()
    res = torch.empty(ncw, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    assert L.ezrs_decode(c._h, C.c_void_p(d.data_ptr()), 255, 223, None, 0, None, 32, None,
                         C.c_void_p(res.data_ptr()), None, 0, None, 0, ncw, C.c_void_p(s)) == 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(res.cpu().numpy(), exp)
    assert res.cpu().numpy()[17] == 3
    np.testing.assert_array_equal(d.cpu().numpy(), good)
