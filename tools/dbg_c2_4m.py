"""Diagnose C2 encode at 4M codewords: encode random rows, decode them clean, and report which
codewords come back flagged (tile index, row in tile, launch chunk), plus a parity check of a
sample against the oracle.  Usage: python tools/dbg_c2_4m.py [ncw]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ezpwd-reed-solomon_amd"))
import ezrs  # noqa: E402

ncw = int(sys.argv[1]) if len(sys.argv) > 1 else 4 << 20
c = ezrs.Codec.rs(255, 223)
gen = torch.Generator(device="cuda").manual_seed(0x5EED0004)
cw = torch.randint(0, 256, (ncw, 255), generator=gen, device="cuda", dtype=torch.int32).to(torch.uint8)
c.encode(cw, 223)
torch.cuda.synchronize()
r = c.decode(cw.clone(), 223)
torch.cuda.synchronize()
bad = torch.nonzero(r != 0).flatten().cpu().numpy()
print(f"ncw {ncw}: {len(bad)} codewords not clean after encode ({100.0 * len(bad) / ncw:.3f} %)")
if len(bad):
    t = bad // 256
    print(" tiles:", np.unique(t)[:40], "... n tiles", len(np.unique(t)))
    print(" row-in-tile histogram (by 32):", np.bincount((bad % 256) // 32, minlength=8))
    print(" chunk of 2048 histogram (first 20):", np.unique(bad // 2048, return_counts=True)[1][:20])
    print(" first bad:", bad[:20])
    print(" tile // 512 histogram:", np.bincount(t // 512)[:40])
