"""Phil Karn's libfec RS ABI over the engine (include/ezrs_fec.h, libezrs_fec.so) against libfec's own
outputs (tests/golden/karn_sem.npz, tests/golden/make_karn_sem_fixtures.py): every Tab row symbol
size of phil-karn/rstest.c:26-50, shortened codewords, erasures in the pad and overwhelmed words
(where Karn's decoder and ezpwd's differ).  Parity, results, corrected rows and positions -- in
libfec's order, full NN frame -- are compared exactly, through the batch forms, the single-codeword
calls and the device-batch API in Karn mode (ezrs_set_semantics)."""
import ctypes as C
import os

import numpy as np
import pytest

import karn_sem_util as KS

pytestmark = pytest.mark.gpu

CASES = KS.cases()
_vp, _sz, _i = C.c_void_p, C.c_size_t, C.c_int


@pytest.fixture(scope="module")
def fec():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ezrs
    L = C.CDLL(os.path.join(os.path.dirname(ezrs.LIB_PATH), "libezrs_fec.so"))
    for f in ("init_rs_char", "init_rs_int"):
        getattr(L, f).restype = _vp
        getattr(L, f).argtypes = [_i] * 6
    for f in ("free_rs_char", "free_rs_int"):
        getattr(L, f).argtypes = [_vp]
    for f in ("encode_rs_char_batch", "encode_rs_int_batch"):
        getattr(L, f).argtypes = [_vp, _vp, _sz, _vp, _sz, _sz]
    for f in ("decode_rs_char_batch", "decode_rs_int_batch"):
        getattr(L, f).argtypes = [_vp, _vp, _sz, _vp, _sz, _vp, _vp, _sz]
    L.encode_rs_char.argtypes = [_vp, _vp, _vp]
    L.decode_rs_char.argtypes = [_vp, _vp, _vp, _i]
    L.encode_rs_int.argtypes = [_vp, _vp, _vp]
    L.decode_rs_int.argtypes = [_vp, _vp, _vp, _i]
    for f in ("encode_rs_8", "encode_rs_ccsds"):
        getattr(L, f).argtypes = [_vp, _vp, _i]
    for f in ("decode_rs_8", "decode_rs_ccsds"):
        getattr(L, f).argtypes = [_vp, _vp, _i, _i]
    L.pad_rs_char.restype = _vp
    L.pad_rs_char.argtypes = [_vp, _i]
    L.ezrs_fec_codec.restype = _vp
    L.ezrs_fec_codec.argtypes = [_vp]
    return L


def _p(a):
    return a.ctypes.data_as(_vp)


def _check_positions(res, pos, exp, nr):
    for k in np.nonzero(res > 0)[0]:
        np.testing.assert_array_equal(pos[k, :res[k]], exp[k, :res[k]], err_msg=f"positions cw {k}")


@pytest.mark.parametrize("case", [c for c in CASES if c["kind"] in ("char", "int")], ids=lambda c: c["id"])
def test_batch_forms_match_libfec(fec, case):
    m, poly, fcr, prim, nr = case["params"]
    pad, ints = case["pad"], case["kind"] == "int"
    init = fec.init_rs_int if ints else fec.init_rs_char
    rs = init(m, poly, fcr, prim, nr, pad)
    assert rs, "init failed"
    try:
        dt = np.uint32 if ints else np.uint8
        data = case["data"].astype(dt)
        ncw, K = data.shape
        par = np.zeros((ncw, nr), dt)
        enc = fec.encode_rs_int_batch if ints else fec.encode_rs_char_batch
        assert enc(rs, _p(data), K, _p(par), nr, ncw) == 0
        np.testing.assert_array_equal(par, case["parity"].astype(dt))
        rows = case["dec_in"].astype(dt)
        eras = case["dec_eras"].astype(np.int32).copy()
        neras = case["dec_neras"].astype(np.int32)
        res = np.zeros(ncw, np.int32)
        dec = fec.decode_rs_int_batch if ints else fec.decode_rs_char_batch
        assert dec(rs, _p(rows), rows.shape[1], _p(eras), nr, _p(neras), _p(res), ncw) == 0
        np.testing.assert_array_equal(res, case["dec_result"])
        np.testing.assert_array_equal(rows, case["dec_out"].astype(dt))
        _check_positions(res, eras, case["dec_positions"], nr)
    finally:
        (fec.free_rs_int if ints else fec.free_rs_char)(rs)


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["id"])
def test_single_codeword_calls_match_libfec(fec, case):
    """encode_rs_* / decode_rs_* one codeword at a time (48 per case, every Karn entry point)."""
    m, poly, fcr, prim, nr = case["params"]
    pad, kind = case["pad"], case["kind"]
    ints = kind == "int"
    dt = np.uint32 if ints else np.uint8
    n = min(48, case["data"].shape[0])
    rs = None
    if kind in ("char", "int"):
        rs = (fec.init_rs_int if ints else fec.init_rs_char)(m, poly, fcr, prim, nr, pad)
        assert rs
    try:
        for k in range(n):
            d = np.ascontiguousarray(case["data"][k].astype(dt))
            p = np.zeros(nr, dt)
            if kind == "char":
                fec.encode_rs_char(rs, _p(d), _p(p))
            elif kind == "int":
                fec.encode_rs_int(rs, _p(d), _p(p))
            else:
                getattr(fec, f"encode_rs_{kind}")(_p(d), _p(p), pad)
            np.testing.assert_array_equal(p, case["parity"][k].astype(dt), err_msg=f"parity cw {k}")
            row = np.ascontiguousarray(case["dec_in"][k].astype(dt))
            ne = int(case["dec_neras"][k])
            ep = np.zeros(nr, np.int32)
            ep[:ne] = case["dec_eras"][k, :ne]
            if kind == "char":
                r = fec.decode_rs_char(rs, _p(row), _p(ep), ne)
            elif kind == "int":
                r = fec.decode_rs_int(rs, _p(row), _p(ep), ne)
            else:
                r = getattr(fec, f"decode_rs_{kind}")(_p(row), _p(ep), ne, pad)
            assert r == case["dec_result"][k], f"result cw {k}"
            np.testing.assert_array_equal(row, case["dec_out"][k].astype(dt), err_msg=f"row cw {k}")
            if r > 0:
                np.testing.assert_array_equal(ep[:r], case["dec_positions"][k, :r], err_msg=f"positions cw {k}")
    finally:
        if rs:
            (fec.free_rs_int if ints else fec.free_rs_char)(rs)


@pytest.mark.parametrize("case", [c for c in CASES if c["params"][0] == 8], ids=lambda c: c["id"])
def test_device_batches_in_karn_mode(fec, case):
    """ezrs_decode on device tensors of a Karn-mode codec (ezrs.Codec.semantics = 'karn'): the
    plane-sliced / bit-sliced syndrome kernels and the GF(2^8) error path under Karn's rules."""
    import torch
    import ezrs
    m, poly, fcr, prim, nr = case["params"]
    c = ezrs.Codec(m, poly, fcr, prim, nr, dual=case["kind"] == "ccsds")
    c.semantics = "karn"
    assert c.semantics == "karn"
    K = case["data"].shape[1]
    rows = torch.from_numpy(case["dec_in"].copy()).cuda()
    eras = torch.from_numpy(case["dec_eras"].astype(np.int32)).cuda()
    neras = torch.from_numpy(case["dec_neras"].astype(np.int32)).cuda()
    pos = torch.zeros((rows.shape[0], nr), dtype=torch.int32, device="cuda")
    res = c.decode(rows, K, None, eras=eras, neras=neras, positions=pos)
    torch.cuda.synchronize()
    res = res.cpu().numpy()
    np.testing.assert_array_equal(res, case["dec_result"])
    np.testing.assert_array_equal(rows.cpu().numpy(), case["dec_out"])
    _check_positions(res, pos.cpu().numpy(), case["dec_positions"], nr)


def test_pad_rs_changes_the_frame(fec):
    """pad_rs_char (phil-karn/pad_rs.c): rejects a pad that leaves no data symbol, else re-pads."""
    rs = fec.init_rs_char(8, 0x11d, 1, 1, 32, 0)
    try:
        assert not fec.pad_rs_char(rs, 223)
        assert fec.pad_rs_char(rs, 100) == rs
        case = next(c for c in CASES if c["kind"] == "char" and c["params"] == (8, 0x11d, 1, 1, 32) and c["pad"])
        assert fec.pad_rs_char(rs, case["pad"]) == rs
        d = np.ascontiguousarray(case["data"][0])
        p = np.zeros(32, np.uint8)
        fec.encode_rs_char(rs, _p(d), _p(p))
        np.testing.assert_array_equal(p, case["parity"][0])
        assert fec.ezrs_fec_codec(rs)
    finally:
        fec.free_rs_char(rs)


@pytest.mark.parametrize("nr", [32, 40])
def test_karn_erasures_checked_after_syndromes(fec, nr):
    """Karn mode checks the syndromes before the erasure positions, as libfec's decode_rs does
    (decode_rs.h:108-132): a clean word with an erasure position >= NN decodes to 0, a corrupted one
    to -1 (libfec's result is undefined there).  ezpwd mode rejects the position first (-1 for both,
    rs_base:1383-1387).  NR 32 runs the plane-sliced path, NR 40 the generic one."""
    import torch
    import ezrs
    K = 255 - nr - 20                                   # shortened: pad 20
    rng = np.random.default_rng(nr)
    clean = torch.from_numpy(rng.integers(0, 256, (8, K + nr)).astype(np.uint8)).cuda()
    eras = torch.zeros((8, nr), dtype=torch.int32, device="cuda")
    eras[:, 0] = 300
    neras = torch.ones(8, dtype=torch.int32, device="cuda")
    for mode in ("karn", "ezpwd"):
        c = ezrs.Codec(8, 0x11d, 1, 1, nr)
        c.semantics = mode
        assert c.kernel_path == ("planeslice" if nr == 32 else "generic")
        c.encode(clean, K)
        rows = clean.clone()
        rows[4:, 3] ^= 0x5A                             # rows 4..7 corrupted
        res = c.decode(rows, K, eras=eras, neras=neras).cpu().numpy()
        torch.cuda.synchronize()
        if mode == "karn":
            np.testing.assert_array_equal(res, [0] * 4 + [-1] * 4)
        else:
            np.testing.assert_array_equal(res, [-1] * 8)
        assert torch.equal(rows[:4], clean[:4])


@pytest.mark.parametrize("case", [c for c in CASES if c["params"][0] == 8 and c["kind"] != "ccsds"],
                         ids=lambda c: c["id"])
def test_device_karn_corrections(fec, case):
    """Corrections (`corr`) of a Karn-mode device decode: for every root in the data or parity the
    value XORed into the row (libfec's in/out difference at that position; an entry is left alone
    where the error value is zero), for a root in the pad (counted but not corrected,
    decode_rs.h:277-289) exactly zero (include/ezrs.h documents it), and left alone
    where a data / parity root's error value is zero."""
    import torch
    import ezrs
    m, poly, fcr, prim, nr = case["params"]
    c = ezrs.Codec(m, poly, fcr, prim, nr)
    c.semantics = "karn"
    K = case["data"].shape[1]
    pad = case["pad"]
    rows = torch.from_numpy(case["dec_in"].copy()).cuda()
    eras = torch.from_numpy(case["dec_eras"].astype(np.int32)).cuda()
    neras = torch.from_numpy(case["dec_neras"].astype(np.int32)).cuda()
    pos = torch.zeros((rows.shape[0], nr), dtype=torch.int32, device="cuda")
    corr = torch.full((rows.shape[0], nr), 0xEE, dtype=torch.uint8, device="cuda")
    res = c.decode(rows, K, None, eras=eras, neras=neras, positions=pos, corr=corr).cpu().numpy()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(res, case["dec_result"])
    pos, corr = pos.cpu().numpy().view(np.uint32), corr.cpu().numpy()
    diff = case["dec_in"] ^ case["dec_out"]
    npad = 0
    for k in np.nonzero(res > 0)[0]:
        for j in range(res[k]):
            p = int(pos[k, j])                          # full-frame position
            if p < pad:
                npad += 1
                assert corr[k, j] == 0, f"cw {k} root {j} in the pad"   # include/ezrs.h: zero
            else:                                       # (0xEE also: a zero error value, not written)
                d = diff[k, p - pad]
                assert corr[k, j] == d or (corr[k, j] == 0xEE and d == 0), f"cw {k} root {j}"
    print(f"{case['id']}: {int((res > 0).sum())} corrected words, {npad} pad roots")
