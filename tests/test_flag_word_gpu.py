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


def test_flag_word_split_launches_and_shard_batches(torch):
    """several syndrome launches of one call share the call's flag number (launches
    split with set_launch_rows, and shard batches, whose launches hold whole shards): a codeword
    flagged only by a later launch must still reach the error path, in alternating clean and
    corrupted calls on one codec and one stream."""
    import ezrs
    c = ezrs.Codec.rs(255, 223)
    oc = O.Codec(*O.rs_params(255, 223))
    rng = np.random.default_rng(0xF1A9)
    try:
        c.set_launch_rows(700)                  # a 3000-codeword call -> 5 syndrome launches
        ncw = 3000
        clean = rng.integers(0, 256, (ncw, 255)).astype(np.uint8)
        oc.encode_batch(clean, 223, None, nthreads=8)
        for it, kind in enumerate(("clean", "bad", "clean", "bad", "bad", "clean")):
            cw = clean.copy()
            if kind == "bad":                   # only rows of the last launches
                for k in rng.choice(np.arange(2100, ncw), 4, replace=False):
                    cw[k, rng.choice(255, 3, replace=False)] ^= rng.integers(1, 256, 3).astype(np.uint8)
            exp = cw.copy()
            exp_r = oc.decode_batch(exp, 223, None, nthreads=8)
            dev = torch.from_numpy(cw).cuda()
            r = c.decode(dev, 223).cpu().numpy()
            torch.cuda.synchronize()
            np.testing.assert_array_equal(r, exp_r, err_msg=f"call {it} ({kind})")
            np.testing.assert_array_equal(dev.cpu().numpy(), exp, err_msg=f"call {it} ({kind})")
        # shard batch: 200 shards of 2000 data bytes (9 codewords each, the last 216 bytes long)
        S, ns = 2000, 200
        R = c.shard_codewords(S)
        enc_len = c.shard_encoded_len(S)
        assert (R, enc_len) == (9, 2000 + 9 * 32)
        buf = torch.from_numpy(rng.integers(0, 256, (ns, enc_len)).astype(np.uint8)).cuda()
        c.encode_shards(buf, S)
        good = buf.clone()
        for it, kind in enumerate(("bad", "clean", "bad", "clean")):
            bad_cw = []
            if kind == "bad":
                h = good.cpu().numpy()
                for q in rng.choice(np.arange(150, ns), 3, replace=False):
                    j = int(rng.integers(0, R))
                    span = (223 if j < R - 1 else S - (R - 1) * 223) + 32
                    locs = j * 255 + rng.choice(span, 4, replace=False)
                    h[q, locs] ^= rng.integers(1, 256, 4).astype(np.uint8)
                    bad_cw.append(q * R + j)
                buf = torch.from_numpy(h).cuda()
            else:
                buf = good.clone()
            r = c.decode_shards(buf, S).cpu().numpy()
            torch.cuda.synchronize()
            exp_r = np.zeros(ns * R, np.int32)
            exp_r[bad_cw] = 4
            np.testing.assert_array_equal(r, exp_r, err_msg=f"shard call {it} ({kind})")
            assert torch.equal(buf, good), f"shard call {it} ({kind})"
    finally:
        c.set_launch_rows(0)
