"""The plane-sliced decode's flag word (ezrs_capi.hip dispatch_decode, DecodeArgs::flag_word): the
syndrome kernel stores the call's number into the workspace when it flags a codeword, and the error
path skips its screen when the word holds another number.  Clean and corrupted batches alternate on
one codec and one stream (one workspace), in both orders, with and without erasures, so a stale
word from an earlier call can neither hide this call's errors nor be mistaken for them."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def test_alternating_clean_and_corrupted_calls(torch):
    import ezrs
    c = ezrs.Codec.rs(255, 223)
    assert c.kernel_path == "planeslice"
    oc = O.Codec(*O.rs_params(255, 223))
    rng = np.random.default_rng(7)
    ncw = 3000
    clean = rng.integers(0, 256, (ncw, 255)).astype(np.uint8)
    oc.encode_batch(clean, 223, None, nthreads=8)
    for it, kind in enumerate(("clean", "bad", "bad", "clean", "bad", "clean", "clean", "eras", "clean")):
        cw = clean.copy()
        eras = neras = None
        if kind != "clean":
            rows = rng.choice(ncw, 5 if kind == "bad" else 0, replace=False)
            for k in rows:
                locs = rng.choice(255, 3, replace=False)
                cw[k, locs] ^= rng.integers(1, 256, 3).astype(np.uint8)
        if kind == "eras":                      # erasures flag codewords the syndromes do not
            eras = np.zeros((ncw, 32), np.uint32)
            neras = np.zeros(ncw, np.uint32)
            neras[[3, 1000]] = 1
            eras[[3, 1000], 0] = [17, 200]
        exp = cw.copy()
        exp_r = oc.decode_batch(exp, 223, None, eras=eras, neras=neras, nthreads=8)
        dev = torch.from_numpy(cw).cuda()
        kw = {}
        if eras is not None:
            kw = dict(eras=torch.from_numpy(eras.view(np.int32)).cuda(),
                      neras=torch.from_numpy(neras.view(np.int32)).cuda())
        r = c.decode(dev, 223, **kw).cpu().numpy()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(r, exp_r, err_msg=f"call {it} ({kind})")
        np.testing.assert_array_equal(dev.cpu().numpy(), exp, err_msg=f"call {it} ({kind})")
        if kind == "bad":
            assert (r == 3).sum() == 5
