"""Host-side enqueue cost of the C2 calls against their GPU time: enqueue K encode (or decode, or
encode+decode) calls without synchronising, then wait; prints host ms per call (the Python ->
ctypes -> HIP launch path) and the wall ms per call including the GPU drain."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ezpwd-reed-solomon_amd"))
import ezrs  # noqa: E402

c = ezrs.Codec.rs(255, 223)
ncw = 1 << 20
cw = torch.randint(0, 256, (ncw, 255), device="cuda", dtype=torch.int32).to(torch.uint8)
res = torch.empty(ncw, dtype=torch.int32, device="cuda")
c.reserve(ncw)
st = torch.cuda.current_stream()
K = 200
for name, fns in (("encode", [lambda: c.encode(cw, 223, stream=st)]),
                  ("decode", [lambda: c.decode(cw, 223, result=res, stream=st)]),
                  ("pair", [lambda: c.encode(cw, 223, stream=st), lambda: c.decode(cw, 223, result=res, stream=st)])):
    for _ in range(10):
        for f in fns:
            f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        for f in fns:
            f()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name}: host enqueue {1e3 * (t1 - t0) / K:.4f} ms/iter, wall {1e3 * (t2 - t0) / K:.4f} ms/iter")
# raw ctypes cost without the Python wrapper checks
L = ezrs.lib()
import ctypes as C
h, p = c._h, C.c_void_p(cw.data_ptr())
sp = C.c_void_p(st.cuda_stream)
t0 = time.perf_counter()
for _ in range(K):
    L.ezrs_encode_rows(h, p, 255, 223, ncw, sp)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"raw ctypes encode: host {1e3 * (t1 - t0) / K:.4f} ms/call, wall {1e3 * (t2 - t0) / K:.4f}")
