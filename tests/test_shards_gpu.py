"""Shard batches (ezrs_encode_shards / ezrs_decode_shards): S-byte shards in the rsencode layout
(rsencode.C:93-163 -- chunks of `chunk` data symbols each followed by its parity, the last chunk
shortened), the whole batch in one call.  Every codeword is checked bit-exactly against the oracle,
which encodes / decodes the same rows one uniform-length batch at a time (full chunks, then the
shortened tails)."""
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


def _geom(S, chunk, nr):
    R = -(-S // chunk)
    tail = S - (R - 1) * chunk
    return R, tail, S + R * nr


def _rows(buf, S, chunk, nr):
    """Views of the full rows ([nshards*(R-1), chunk+nr]) and tail rows ([nshards, tail+nr])
    of a shard buffer [nshards, pitch] (copies, in codeword order)."""
    R, tail, enc = _geom(S, chunk, nr)
    ns = buf.shape[0]
    step = chunk + nr
    full = np.stack([buf[:, j * step:(j + 1) * step] for j in range(R - 1)], axis=1) \
        if R > 1 else np.zeros((ns, 0, step), buf.dtype)
    tl = buf[:, (R - 1) * step:(R - 1) * step + tail + nr].copy()
    return full.reshape(-1, step).copy(), tl


def _put(buf, full, tl, S, chunk, nr):
    R, tail, _ = _geom(S, chunk, nr)
    ns = buf.shape[0]
    step = chunk + nr
    f = full.reshape(ns, R - 1, step)
    for j in range(R - 1):
        buf[:, j * step:(j + 1) * step] = f[:, j]
    buf[:, (R - 1) * step:(R - 1) * step + tail + nr] = tl


def _codeword_order(full_res, tail_res, ns, R):
    """Per-codeword values (shard-major) from the full-row and tail-row results."""
    out = np.zeros((ns, R) + full_res.shape[1:], full_res.dtype)
    if R > 1:
        out[:, :R - 1] = full_res.reshape((ns, R - 1) + full_res.shape[1:])
    out[:, R - 1] = tail_res
    return out.reshape((ns * R,) + full_res.shape[1:])


CASES = [
    # (n, k, S, chunk, nshards, pad)
    (255, 223, 1024, 223, 300, 0),        # 1 KiB shards: 5 codewords, the last 132 symbols
    (255, 223, 1024, 223, 257, 7),        # padded shard pitch
    (255, 223, 16384, 223, 20, 0),
    (255, 223, 223, 223, 600, 0),         # one full codeword per shard (no shortened row)
    (255, 223, 100, 223, 700, 3),         # one shortened codeword per shard
    (255, 223, 447, 223, 400, 0),         # 3 rows, tail of 1 symbol
    (255, 223, 1000, 200, 300, 0),        # chunks shorter than the load: every row shortened
    (255, 239, 4096, 239, 90, 0),
    (255, 251, 2000, 251, 150, 1),
]


@pytest.mark.parametrize("n,k,S,chunk,ns,pad", CASES)
def test_shards_vs_oracle(torch, n, k, S, chunk, ns, pad):
    import ezrs
    c = ezrs.Codec.rs(n, k)
    oc = O.Codec(*O.rs_params(n, k))
    nr = n - k
    R, tail, enc = _geom(S, chunk, nr)
    assert c.shard_codewords(S, chunk) == R and c.shard_encoded_len(S, chunk) == enc
    pitch = enc + pad
    rng = np.random.default_rng(S * 7 + chunk + ns)
    host = rng.integers(0, 256, (ns, pitch)).astype(np.uint8)
    dev = torch.from_numpy(host.copy()).cuda()
    c.encode_shards(dev, S, chunk)
    full, tl = _rows(host, S, chunk, nr)
    oc.encode_batch(full, chunk)
    oc.encode_batch(tl, tail)
    exp = host.copy()
    _put(exp, full, tl, S, chunk, nr)
    got = dev.cpu().numpy()
    np.testing.assert_array_equal(got[:, :enc], exp[:, :enc], err_msg="shard encode")
    np.testing.assert_array_equal(got[:, enc:], host[:, enc:], err_msg="pad bytes touched")

    # decode: 0..nr/2 symbol errors in random codewords (tails included), one overwhelmed row
    bad = exp.copy()
    nerr = rng.integers(0, nr // 2 + 1, ns * R)
    nerr[rng.integers(0, ns * R)] = nr // 2 + 3
    step = chunk + nr
    for kk in np.nonzero(nerr)[0]:
        s, j = divmod(int(kk), R)
        L = (chunk if j < R - 1 else tail) + nr
        locs = rng.choice(L, min(int(nerr[kk]), L), replace=False)
        bad[s, j * step + locs] ^= rng.integers(1, 256, len(locs)).astype(np.uint8)
    dev = torch.from_numpy(bad.copy()).cuda()
    pos = torch.zeros((ns * R, nr), dtype=torch.int32, device="cuda")
    res = c.decode_shards(dev, S, chunk, positions=pos)
    full, tl = _rows(bad, S, chunk, nr)
    pf = np.zeros((full.shape[0], nr), np.uint32)
    pt = np.zeros((tl.shape[0], nr), np.uint32)
    rf = oc.decode_batch(full, chunk, positions=pf) if R > 1 else np.zeros(0, np.int32)
    rt = oc.decode_batch(tl, tail, positions=pt)
    exp_d = bad.copy()
    _put(exp_d, full, tl, S, chunk, nr)
    exp_r = _codeword_order(rf, rt, ns, R)
    np.testing.assert_array_equal(res.cpu().numpy(), exp_r, err_msg="shard decode results")
    np.testing.assert_array_equal(dev.cpu().numpy(), exp_d, err_msg="shard decode data")
    exp_p = _codeword_order(pf, pt, ns, R)
    gp = pos.cpu().numpy().view(np.uint32)
    for kk in range(ns * R):
        r = exp_r[kk]
        if r > 0:
            np.testing.assert_array_equal(gp[kk, :r], exp_p[kk, :r], err_msg=f"positions cw {kk}")


def test_shards_erasures_generic_codec(torch):
    """A codec without a sliced path (RS_CCSDS(255,223) dual basis) runs shard batches on the
    per-codeword kernels; erasures index each codeword from its first data symbol."""
    import ezrs
    c = ezrs.Codec.ccsds(223, dual=True)
    oc = O.Codec(*O.ccsds_params(223, True))
    nr, S, chunk, ns = 32, 700, 223, 64
    R, tail, enc = _geom(S, chunk, nr)
    rng = np.random.default_rng(11)
    host = rng.integers(0, 256, (ns, enc)).astype(np.uint8)
    dev = torch.from_numpy(host.copy()).cuda()
    c.encode_shards(dev, S, chunk)
    full, tl = _rows(host, S, chunk, nr)
    oc.encode_batch(full, chunk)
    oc.encode_batch(tl, tail)
    exp = host.copy()
    _put(exp, full, tl, S, chunk, nr)
    np.testing.assert_array_equal(dev.cpu().numpy(), exp)
    # 3 errors + 4 erasures in every codeword
    bad = exp.copy()
    eras = np.zeros((ns * R, nr), np.uint32)
    neras = np.full(ns * R, 4, np.uint32)
    step = chunk + nr
    for kk in range(ns * R):
        s, j = divmod(kk, R)
        L = (chunk if j < R - 1 else tail) + nr
        locs = rng.choice(L, 7, replace=False)
        bad[s, j * step + locs] ^= rng.integers(1, 256, 7).astype(np.uint8)
        eras[kk, :4] = locs[3:]
    dev = torch.from_numpy(bad.copy()).cuda()
    res = c.decode_shards(dev, S, chunk, eras=torch.from_numpy(eras.view(np.int32)).cuda(),
                          neras=torch.from_numpy(neras.view(np.int32)).cuda())
    full, tl = _rows(bad, S, chunk, nr)
    ef = eras.reshape(ns, R, nr)
    rf = oc.decode_batch(full, chunk, eras=ef[:, :R - 1].reshape(-1, nr).copy(),
                         neras=np.full(full.shape[0], 4, np.uint32))
    rt = oc.decode_batch(tl, tail, eras=ef[:, R - 1].copy(), neras=np.full(ns, 4, np.uint32))
    exp_d = bad.copy()
    _put(exp_d, full, tl, S, chunk, nr)
    np.testing.assert_array_equal(res.cpu().numpy(), _codeword_order(rf, rt, ns, R))
    np.testing.assert_array_equal(dev.cpu().numpy(), exp_d)


def test_shards_c2_size_round_trip(torch):
    """~256 MB of 1 KiB shards (the bench's sweep point): encode, corrupt a sample, decode."""
    import ezrs
    c = ezrs.Codec.rs(255, 223)
    S, nr = 1024, 32
    R, tail, enc = _geom(S, 223, nr)
    ns = (256 << 20) // S
    g = torch.Generator(device="cuda").manual_seed(5)
    dev = torch.randint(0, 256, (ns, enc), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
    c.encode_shards(dev, S)
    ref = dev.clone()
    res = c.decode_shards(dev, S)
    assert int((res != 0).sum()) == 0
    # 16 errors in the tail codeword and 5 in the first of every 97th shard
    idx = torch.arange(0, ns, 97, device="cuda")
    col_t = (R - 1) * (223 + nr) + torch.arange(16, device="cuda") * 7
    col_f = torch.arange(5, device="cuda") * 31
    for col in (col_t, col_f):
        dev[idx[:, None], col[None, :]] ^= 0x5A
    res = c.decode_shards(dev, S)
    r = res.view(ns, R)
    assert int((r[idx, R - 1] != 16).sum()) == 0 and int((r[idx, 0] != 5).sum()) == 0
    assert int((res != 0).sum()) == 2 * len(idx)
    assert torch.equal(dev, ref)
