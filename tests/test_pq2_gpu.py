"""Full-length RS(255,223) rows at pitch 255 -- the geometry the double-buffered tile kernel k_pq2
takes (ezrs_ps.hip) -- against the oracle on every codeword: encode parity, and decode results,
positions and corrected rows under random error loads (clean, correctable, overwhelmed).  Batch sizes
off the 256-codeword tile and the 16-byte piece grid exercise the partial last tile and the re-read of
the piece that crosses the batch's end; a base offset by one byte takes the k_pq_lin fallback."""
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


@pytest.mark.parametrize("ncw,offset", [(1, 0), (7, 0), (255, 0), (257, 0), (4096, 0), (4173, 0),
                                        (65536 + 13, 0), (1000, 1), (3 * 2048 + 5, 16)])
def test_full_length_vs_oracle(torch, ncw, offset):
    import ezrs
    c = ezrs.Codec.rs(255, 223)
    oc = O.Codec(*O.rs_params(255, 223))
    rng = np.random.default_rng(ncw * 7 + offset)
    data = rng.integers(0, 256, (ncw, 255)).astype(np.uint8)
    ref = data.copy()
    oc.encode_batch(ref, 223, None, nthreads=8)
    # a byte buffer with the batch at `offset` (offset 1: an unaligned base)
    buf = torch.zeros(ncw * 255 + 64, dtype=torch.uint8, device="cuda")
    dev = buf[offset:offset + ncw * 255].view(ncw, 255)
    dev.copy_(torch.from_numpy(data).cuda())
    c.encode(dev, 223)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(dev.cpu().numpy(), ref)
    assert int(buf[:offset].count_nonzero()) == 0 and int(buf[offset + ncw * 255:].count_nonzero()) == 0
    # errors: loads 0 .. 20 per codeword (past the 16-error capacity for some)
    load = rng.integers(0, 21, ncw)
    load[::3] = 0
    cw = ref.copy()
    for k in range(ncw):
        m = int(load[k])
        if m:
            locs = rng.choice(255, m, replace=False)
            cw[k, locs] ^= rng.integers(1, 256, m).astype(np.uint8)
    exp = cw.copy()
    exp_pos = np.zeros((ncw, 32), np.uint32)
    exp_r = oc.decode_batch(exp, 223, None, positions=exp_pos, nthreads=8)
    dev.copy_(torch.from_numpy(cw).cuda())
    pos = torch.zeros((ncw, 32), dtype=torch.int32, device="cuda")
    r = c.decode(dev, 223, positions=pos)
    torch.cuda.synchronize()
    r = r.cpu().numpy()
    np.testing.assert_array_equal(r, exp_r)
    np.testing.assert_array_equal(dev.cpu().numpy(), exp)
    pos = pos.cpu().numpy().view(np.uint32)
    for k in np.nonzero(r > 0)[0]:
        np.testing.assert_array_equal(pos[k, :r[k]], exp_pos[k, :r[k]])
    if ncw >= 255:
        assert (r == 0).any() and (r > 0).any()


def test_full_length_clean_large(torch):
    """1M + 37 clean codewords (every workgroup runs several tiles, the last one partial): decode
    returns 0 everywhere; one corrupted symbol in each of the last 300 rows is found and fixed."""
    import ezrs
    c = ezrs.Codec.rs(255, 223)
    ncw = (1 << 20) + 37
    gen = torch.Generator(device="cuda").manual_seed(0x5EED0099)
    cw = torch.randint(0, 256, (ncw, 255), generator=gen, device="cuda", dtype=torch.int32).to(torch.uint8)
    c.encode(cw, 223)
    r = c.decode(cw.clone(), 223)
    torch.cuda.synchronize()
    assert int((r != 0).sum()) == 0
    bad = cw.clone()
    rows = torch.arange(ncw - 300, ncw, device="cuda")
    cols = torch.randint(0, 255, (300,), generator=gen, device="cuda")
    bad[rows, cols] ^= 0x5A
    r = c.decode(bad, 223)
    torch.cuda.synchronize()
    assert int((r[:ncw - 300] != 0).sum()) == 0 and int((r[ncw - 300:] != 1).sum()) == 0
    assert torch.equal(bad, cw)
