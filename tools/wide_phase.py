"""Phase timing of the GF(2^16) error kernel: C4 corruption, decode only, EZRS_WIDE_STOP = 1 (after
the syndrome load), 2 (after Berlekamp-Massey), 4 (after the squarings), 3 (after the root finder), 0 (full)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ezpwd-reed-solomon_amd"))
import ezrs  # noqa: E402

ncw = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
n, k = 65535, 65503
c = ezrs.Codec.rs(n, k)
c.reserve(ncw)
rng = np.random.default_rng(5)
host = rng.integers(0, n + 1, (ncw, n)).astype(np.uint16)
clean = torch.from_numpy(host.view(np.int16)).cuda().view(torch.uint16)
c.encode(clean, k)
torch.cuda.synchronize()
enc = clean.view(torch.int16).cpu().numpy().view(np.uint16)
bad = enc.copy()
eras = np.zeros((ncw, 32), np.uint32)
locs = np.stack([rng.choice(n, 12, replace=False) for _ in range(ncw)])
bad[np.arange(ncw)[:, None], locs] ^= rng.integers(1, n + 1, (ncw, 12)).astype(np.uint16)
eras[:, :4] = locs[:, 8:]
master = torch.from_numpy(bad.view(np.int16)).cuda()
work = torch.empty_like(master)
d_eras = torch.from_numpy(eras.view(np.int32)).cuda()
d_neras = torch.full((ncw,), 4, dtype=torch.int32, device="cuda")
result = torch.empty(ncw, dtype=torch.int32, device="cuda")
for stop in (1, 2, 4, 3, 0):
    os.environ["EZRS_WIDE_STOP"] = str(stop)
    ts = []
    for _ in range(3):
        work.copy_(master)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        c.decode(work.view(torch.uint16), k, eras=d_eras, neras=d_neras, result=result)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ok = bool((result == 12).all())
    print(f"stop={stop} decode ms {min(ts):.3f} (all {['%.3f' % t for t in ts]}) restored={ok}", flush=True)
