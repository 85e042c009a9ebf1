"""C3-shaped decode timing (RS(255,223), 8 errors + 4 erasures per codeword, 1M codewords): the
decode call alone, with a check that the batch is restored."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "ezpwd-reed-solomon_amd"))
import ezrs

ncw, n, k = 1 << 20, 255, 223
c = ezrs.Codec.rs(n, k)
c.reserve(ncw)
rng = np.random.default_rng(3)
host = rng.integers(0, 256, (ncw, n)).astype(np.uint8)
clean = torch.from_numpy(host).cuda()
c.encode(clean, k)
enc = clean.cpu().numpy()
locs = np.argsort(rng.random((ncw, n)), axis=1)[:, :12]
bad = enc.copy()
bad[np.arange(ncw)[:, None], locs] ^= rng.integers(1, 256, (ncw, 12)).astype(np.uint8)
eras = np.zeros((ncw, 32), np.uint32)
eras[:, :4] = locs[:, 8:]
master = torch.from_numpy(bad).cuda()
work = torch.empty_like(master)
d_eras = torch.from_numpy(eras.view(np.int32)).cuda()
d_neras = torch.full((ncw,), 4, dtype=torch.int32, device="cuda")
result = torch.empty(ncw, dtype=torch.int32, device="cuda")
ts = []
for it in range(23):
    work.copy_(master)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    c.decode(work, k, eras=d_eras, neras=d_neras, result=result)
    e1.record()
    torch.cuda.synchronize()
    if it >= 3:
        ts.append(e0.elapsed_time(e1))
ok = bool((result == 12).all()) and torch.equal(work, clean)
print(f"decode_ms={np.mean(ts):.4f} min={np.min(ts):.4f} ok={ok}")
