"""Karn-side pin (BASELINE config C2: "bit-exact vs phil-karn rstest.c").

tests/golden/karn_*.npz hold Phil Karn's libfec outputs (fec-3.0.1 built from the reference's
tarball by oracle/Makefile `karn`; tests/golden/make_karn_fixtures.py):
  karn_rs255_223  encode_rs_char / decode_rs_char, Tab row {8,0x11d,1,1,32} (phil-karn/rstest.c:36)
                  = ezpwd::RS<255,223>
  karn_8          encode_rs_8 / decode_rs_8 (CCSDS polynomial, conventional basis)
                  = ezpwd::RS_CCSDS_CONV<255,223>
  karn_ccsds      encode_rs_ccsds / decode_rs_ccsds (dual basis) = ezpwd::RS_CCSDS<255,223>
The CPU test checks the oracle restatement against them; the GPU test checks the device codec.
Error positions are compared as sets (libfec lists them in Chien-search order).
"""
import os

import numpy as np
import pytest

import golden_util  # noqa: F401  (puts oracle/ on sys.path)
import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = [("karn_rs255_223", O.rs_params(255, 223)),
         ("karn_8", O.ccsds_params(223, dual=False)),
         ("karn_ccsds", O.ccsds_params(223, dual=True))]


@pytest.fixture(scope="module")
def torch():
    import torch as T
    if not T.cuda.is_available():
        pytest.skip("no GPU")
    return T


def _load(name):
    return dict(np.load(os.path.join(HERE, "golden", name + ".npz")))


def _sets(pos, res):
    return [sorted(int(x) for x in pos[i, :max(int(res[i]), 0)]) for i in range(len(res))]


@pytest.mark.parametrize("name,params", CASES)
def test_oracle_matches_karn(name, params):
    f = _load(name)
    oc = O.Codec(*params)
    K = f["data"].shape[1]
    cw = np.concatenate([f["data"], np.zeros_like(f["parity"])], axis=1)
    oc.encode_batch(cw, K)
    np.testing.assert_array_equal(cw[:, K:], f["parity"])
    rows = f["dec_in"].copy()
    eras = f["dec_eras"].astype(np.uint32)
    neras = f["dec_neras"].astype(np.uint32)
    pos = np.zeros((rows.shape[0], 32), np.uint32)
    res = oc.decode_batch(rows, K, None, eras, neras, pos)
    np.testing.assert_array_equal(res, f["dec_result"])
    np.testing.assert_array_equal(rows, f["dec_out"])
    assert _sets(pos, res) == _sets(f["dec_positions"], f["dec_result"])


@pytest.mark.gpu
@pytest.mark.parametrize("name,params", CASES)
def test_device_matches_karn(torch, name, params):
    import ezrs
    f = _load(name)
    c = ezrs.Codec.rs(255, 223) if name == "karn_rs255_223" else ezrs.Codec.ccsds(223, dual=params[5])
    K = f["data"].shape[1]
    cw = torch.from_numpy(np.concatenate([f["data"], np.zeros_like(f["parity"])], axis=1)).cuda()
    c.encode(cw, K)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(cw.cpu().numpy()[:, K:], f["parity"])
    rows = torch.from_numpy(f["dec_in"].copy()).cuda()
    eras = torch.from_numpy(f["dec_eras"].astype(np.int32)).cuda()
    neras = torch.from_numpy(f["dec_neras"].astype(np.int32)).cuda()
    pos = torch.zeros((rows.shape[0], 32), dtype=torch.int32, device="cuda")
    res = c.decode(rows, K, None, eras=eras, neras=neras, positions=pos)
    torch.cuda.synchronize()
    res = res.cpu().numpy()
    np.testing.assert_array_equal(res, f["dec_result"])
    np.testing.assert_array_equal(rows.cpu().numpy(), f["dec_out"])
    assert _sets(pos.cpu().numpy(), res) == _sets(f["dec_positions"], f["dec_result"])
