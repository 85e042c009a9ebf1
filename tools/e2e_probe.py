"""Time the host-memory forms (ezrs_encode_host / ezrs_decode_host) of RS(255,223) separately,
pageable vs pinned, for a few chunk sizes.  Diagnostic for the PCIe-inclusive rate in DESIGN.md."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ezpwd-reed-solomon_amd"))
import numpy as np
import torch
import ezrs

ncw = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
c = ezrs.Codec.rs(255, 223)
h = np.random.default_rng(3).integers(0, 256, (ncw, 255)).astype(np.uint8)
hp = torch.from_numpy(h.copy()).pin_memory().numpy()
for name, buf in (("pageable", h), ("pinned", hp)):
    for chunk in (0, 1 << 15, 1 << 16, 1 << 17):
        c.encode_host(buf, 223, chunk=chunk)
        c.decode_host(buf, 223, chunk=chunk)
        t0 = time.perf_counter(); c.encode_host(buf, 223, chunk=chunk); t1 = time.perf_counter()
        r = c.decode_host(buf, 223, chunk=chunk); t2 = time.perf_counter()
        assert (r == 0).all()
        print(f"{name:8s} chunk={chunk:7d} encode {1e3*(t1-t0):8.2f} ms  decode {1e3*(t2-t1):8.2f} ms"
              f"  -> {ncw*255/(t2-t0)/1e9:.3f} GB/s", flush=True)
# raw copy-engine rates for the same bytes (one pinned buffer, one device buffer)
t = torch.from_numpy(hp)
d = torch.empty_like(t, device="cuda")
for _ in range(2):
    torch.cuda.synchronize(); t0 = time.perf_counter(); d.copy_(t, non_blocking=True); torch.cuda.synchronize()
    t1 = time.perf_counter(); t.copy_(d, non_blocking=True); torch.cuda.synchronize(); t2 = time.perf_counter()
print(f"raw pinned H2D {ncw*255/(t1-t0)/1e9:.2f} GB/s, D2H {ncw*255/(t2-t1)/1e9:.2f} GB/s", flush=True)
