"""Batches split over several plane-sliced launches: ezrs_set_launch_rows lowers a codec's
per-launch codeword cap so a small batch takes the paths a multi-GB one would -- plain batches whose
launches start off the 256-codeword tile grid, short row pitches, and shard batches whose launches
end mid-tile (the byte-store syndrome path).  Every output is compared with the oracle."""
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


def _corrupt(rng, cw, L, nr, ncw):
    eras = np.zeros((ncw, nr), np.uint32)
    neras = np.zeros(ncw, np.uint32)
    load = rng.integers(0, nr + 3, ncw)
    for k in range(ncw):
        m = min(int(load[k]), L)
        locs = rng.choice(L, m, replace=False)
        cw[k, locs] ^= rng.integers(1, 256, m).astype(np.uint8)
        ne = min(int(rng.integers(0, m + 1)), nr)
        eras[k, :ne] = locs[:ne]
        neras[k] = ne
    return eras, neras


@pytest.mark.parametrize("k,L,rows", [(223, 223, 1000), (223, 16, 300), (247, 40, 2049), (251, 200, 5)])
def test_plain_batch_split_vs_oracle(torch, k, L, rows):
    import ezrs
    c = ezrs.Codec.rs(255, k)
    assert c.kernel_path == "planeslice"
    oc = O.Codec(*O.rs_params(255, k))
    nr, ncw = 255 - k, 5003
    rng = np.random.default_rng(k * 31 + L + rows)
    data = rng.integers(0, 256, (ncw, L + nr)).astype(np.uint8)
    ref = data.copy()
    oc.encode_batch(ref, L, None, nthreads=8)
    c.set_launch_rows(rows)
    dev = torch.from_numpy(data).cuda()
    c.encode(dev, L)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dev.cpu().numpy(), ref, err_msg="encode")
    cw = ref.copy()
    eras, neras = _corrupt(rng, cw, L + nr, nr, ncw)
    exp = cw.copy()
    exp_pos = np.zeros((ncw, nr), np.uint32)
    exp_r = oc.decode_batch(exp, L, None, eras, neras, exp_pos, nthreads=8)
    dcw = torch.from_numpy(cw).cuda()
    pos = torch.zeros((ncw, nr), dtype=torch.int32, device="cuda")
    r = c.decode(dcw, L, None, eras=torch.from_numpy(eras.view(np.int32)).cuda(),
                 neras=torch.from_numpy(neras.view(np.int32)).cuda(), positions=pos)
    torch.cuda.synchronize()
    r = r.cpu().numpy()
    np.testing.assert_array_equal(r, exp_r, err_msg="results")
    np.testing.assert_array_equal(dcw.cpu().numpy(), exp, err_msg="corrected rows")
    pos = pos.cpu().numpy().view(np.uint32)
    for kk in np.nonzero(r > 0)[0]:
        np.testing.assert_array_equal(pos[kk, :r[kk]], exp_pos[kk, :r[kk]])
    assert (r == 0).any() and (r > 0).any()


@pytest.mark.parametrize("S,rows", [(1024, 777), (16384, 300), (600, 1)])
def test_shard_batch_split_vs_oracle(torch, S, rows):
    """Shard launches hold whole shards: 777 rows of 1 KiB shards (5 codewords each) = 155 shards
    per launch, so every launch after the first starts mid-tile."""
    import ezrs
    c = ezrs.Codec.rs(255, 223)
    oc = O.Codec(*O.rs_params(255, 223))
    nr, chunk, ns = 32, 223, 400
    R = -(-S // chunk)
    tail = S - (R - 1) * chunk
    enc = S + R * nr
    rng = np.random.default_rng(S + rows)
    host = rng.integers(0, 256, (ns, enc)).astype(np.uint8)
    step = chunk + nr
    c.set_launch_rows(rows)
    dev = torch.from_numpy(host.copy()).cuda()
    c.encode_shards(dev, S, chunk)
    exp = host.copy()
    for j in range(R):
        L = chunk if j < R - 1 else tail
        blk = exp[:, j * step:j * step + L + nr].copy()
        oc.encode_batch(blk, L)
        exp[:, j * step:j * step + L + nr] = blk
    np.testing.assert_array_equal(dev.cpu().numpy(), exp, err_msg="shard encode")
    bad = exp.copy()
    for s in range(ns):
        for j in range(R):
            L = (chunk if j < R - 1 else tail) + nr
            m = int(rng.integers(0, nr // 2 + 2))
            locs = rng.choice(L, min(m, L), replace=False)
            bad[s, j * step + locs] ^= rng.integers(1, 256, len(locs)).astype(np.uint8)
    dev = torch.from_numpy(bad.copy()).cuda()
    res = c.decode_shards(dev, S, chunk).cpu().numpy().reshape(ns, R)
    exp_d = bad.copy()
    for j in range(R):
        L = chunk if j < R - 1 else tail
        blk = exp_d[:, j * step:j * step + L + nr].copy()
        rr = oc.decode_batch(blk, L)
        exp_d[:, j * step:j * step + L + nr] = blk
        np.testing.assert_array_equal(res[:, j], rr, err_msg=f"results, row {j}")
    np.testing.assert_array_equal(dev.cpu().numpy(), exp_d, err_msg="shard decode data")
