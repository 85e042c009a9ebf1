import sys, numpy as np, torch
sys.path[:0] = ["ezpwd-reed-solomon_amd", "oracle"]
import ezrs, oracle as O
c = ezrs.Codec.rs(255, 223); oc = O.Codec(*O.rs_params(255, 223))
rng = np.random.default_rng(255)
for ncw, chunk in ((3000, 1000), (1000, 0), (3000, 0)):
    rows = rng.integers(0, 256, (ncw, 255)).astype(np.uint8)
    par = np.zeros((ncw, 32), np.uint8)
    c.encode_host(rows, 223, par, chunk=chunk)
    exp = rows.copy(); oc.encode_batch(exp, 223)
    bad = np.nonzero((par != exp[:, 223:]).any(axis=1))[0]
    print("host", ncw, chunk, "bad rows:", bad[:20], len(bad))
    # device, separate parity
    d = torch.from_numpy(rows).cuda(); p = torch.zeros((ncw, 32), dtype=torch.uint8, device="cuda")
    c.encode(d, 223, p); torch.cuda.synchronize()
    bad = np.nonzero((p.cpu().numpy() != exp[:, 223:]).any(axis=1))[0]
    print("dev sep", ncw, "bad rows:", bad[:20], len(bad))
    d2 = torch.from_numpy(rows.copy()).cuda(); c.encode(d2, 223); torch.cuda.synchronize()
    bad = np.nonzero((d2.cpu().numpy() != exp).any(axis=1))[0]
    print("dev rows", ncw, "bad rows:", bad[:20], len(bad))
