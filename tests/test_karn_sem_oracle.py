"""The oracle's Karn mode (oracle/ezrs_oracle.c decode_symbols with ezo_set_karn) against libfec's own
outputs (tests/golden/karn_sem.npz): parity, results, corrected rows and positions in libfec's
order, for shortened codes, erasures in the pad and overwhelmed words -- the cases where Karn's and
ezpwd's decoders differ (fec-3.0.1/decode_rs.h:71-298 vs rs_base:1335-1718)."""
import numpy as np
import pytest

import golden_util  # noqa: F401  (puts oracle/ on sys.path)
import karn_sem_util as KS
import oracle as O

CASES = KS.cases()


@pytest.mark.parametrize("case", CASES, ids=[c["id"] for c in CASES])
def test_oracle_karn_mode_matches_libfec(case):
    m, poly, fcr, prim, nr = case["params"]
    oc = O.Codec(m, poly, fcr, prim, nr, dual=case["kind"] == "ccsds", karn=True)
    K = case["data"].shape[1]
    dt = oc.dtype
    cw = np.concatenate([case["data"], np.zeros_like(case["parity"])], axis=1).astype(dt)
    oc.encode_batch(cw, K)
    np.testing.assert_array_equal(cw[:, K:], case["parity"].astype(dt))
    rows = case["dec_in"].astype(dt)
    eras = case["dec_eras"].astype(np.uint32)
    neras = case["dec_neras"].astype(np.uint32)
    pos = np.zeros((rows.shape[0], nr), np.uint32)
    res = oc.decode_batch(rows, K, None, eras, neras, pos)
    np.testing.assert_array_equal(res, case["dec_result"])
    np.testing.assert_array_equal(rows, case["dec_out"].astype(dt))
    exp = case["dec_positions"]
    for k in np.nonzero(res > 0)[0]:
        np.testing.assert_array_equal(pos[k, :res[k]], exp[k, :res[k]].astype(np.uint32), err_msg=f"cw {k}")
    # the cases that make Karn mode necessary are present
    assert (res >= 0).any()
