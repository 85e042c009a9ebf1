"""Multi-process CPU tests of the sharded batch path (gloo, world size 2): the per-rank ranges
cover the batch, each rank's shard encodes and decodes independently, and the concatenated result
equals the single-process result; the only collectives are the timing max and the count sum.
The oracle stands in for the device codec here (no GPU on this host)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

import shard


def test_shard_range_covers():
    for ncw in (0, 1, 7, 1000, 1 << 20):
        for world in range(1, 9):
            rs = [shard.shard_range(ncw, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == ncw
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            sizes = [hi - lo for lo, hi in rs]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def test_single_process_reductions_are_identity():
    assert shard.max_over_ranks(3.5) == 3.5
    assert shard.sum_over_ranks([1, 2]) == [1, 2]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch():
    rng = np.random.default_rng(99)
    return rng.integers(0, 256, (3001, 255)).astype(np.uint8)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        oc = O.Codec(*O.rs_params(255, 223))
        data = _batch()
        lo, hi = shard.shard_range(len(data), world, rank)
        part = data[lo:hi].copy()
        oc.encode_batch(part, 223)
        part[::5, 17] ^= 0x5A                       # one symbol error in every fifth codeword
        res = oc.decode_batch(part, 223)
        t = shard.max_over_ranks(float(rank + 1))
        counts = shard.sum_over_ranks([int((res == 0).sum()), int((res == 1).sum()), hi - lo])
        q.put((rank, lo, hi, part.tobytes(), res.tobytes(), t, counts))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_sharding():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    import oracle as O
    oc = O.Codec(*O.rs_params(255, 223))
    ref = _batch()
    oc.encode_batch(ref, 223)
    cw = np.concatenate([np.frombuffer(o[3], np.uint8).reshape(-1, 255) for o in out])
    res = np.concatenate([np.frombuffer(o[4], np.int32) for o in out])
    np.testing.assert_array_equal(cw, ref)           # every shard corrected back to the encoding
    assert out[0][2] == out[1][1] and out[1][2] == len(ref)
    assert all(o[5] == 2.0 for o in out)              # max over ranks
    nfix = sum(((hi - lo) + 4) // 5 for _, lo, hi, *_ in out)
    assert all(o[6] == [len(ref) - nfix, nfix, len(ref)] for o in out)
    assert (res >= 0).all()
