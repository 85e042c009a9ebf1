"""C4-shaped timing (RS(65535,65503), 8 errors + 4 erasures per codeword, bench.py's c4 load)
generated on the device: encode and decode calls (HIP events around each, the batch restored from a
master copy before each decode), with a check that every result is 12 and the batch is restored.
The library is the default one or EZRS_LIB_VARIANT's.  Usage: c4_decode_time.py [ncw] [reps]"""
import os, sys, time
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "ezpwd-reed-solomon_amd"))
import ezrs

ncw = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n, k = 65535, 65503
c = ezrs.Codec.rs(n, k)
c.reserve(ncw)
gen = torch.Generator(device="cuda").manual_seed(4)
clean = torch.randint(-32768, 32768, (ncw, n), generator=gen, device="cuda", dtype=torch.int32).to(torch.int16)
c.encode(clean.view(torch.uint16), k)
# 12 distinct positions per codeword: sorted uniforms spread over n - 11, plus 0..11
pos = (torch.sort(torch.rand((ncw, 12), generator=gen, device="cuda"), dim=1).values
       * (n - 11)).to(torch.int64) + torch.arange(12, device="cuda")
pos = pos.gather(1, torch.argsort(torch.rand((ncw, 12), generator=gen, device="cuda"), dim=1))
val = torch.randint(1, 65536, (ncw, 12), generator=gen, device="cuda", dtype=torch.int32)
master = clean.clone()
flat = master.view(-1)
idx = (torch.arange(ncw, device="cuda")[:, None] * n + pos).reshape(-1)
flat[idx] = (flat[idx].to(torch.int32) ^ val.reshape(-1)).to(torch.int16)
eras = torch.zeros((ncw, 32), dtype=torch.int32, device="cuda")
eras[:, :4] = pos[:, 8:].to(torch.int32)
neras = torch.full((ncw,), 4, dtype=torch.int32, device="cuda")
work = torch.empty_like(master)
res = torch.empty(ncw, dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
t0 = time.time()
while time.time() - t0 < 0.5:
    work.copy_(master)
    c.decode(work.view(torch.uint16), k, eras=eras, neras=neras, result=res)
    torch.cuda.synchronize()
ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(reps)]
for e in ev:
    work.copy_(master)
    e[0].record()
    c.encode(clean.view(torch.uint16), k)
    e[1].record()
    c.decode(work.view(torch.uint16), k, eras=eras, neras=neras, result=res)
    e[2].record()
torch.cuda.synchronize()
enc = sum(e[0].elapsed_time(e[1]) for e in ev) / reps
dec = sum(e[1].elapsed_time(e[2]) for e in ev) / reps
ok = bool((res == 12).all()) and torch.equal(work, clean)
print(f"ncw={ncw} encode_ms={enc:.4f} decode_ms={dec:.4f} ok={ok} "
      f"variant={os.path.basename(os.environ.get('EZRS_LIB_VARIANT', 'default'))}", flush=True)
