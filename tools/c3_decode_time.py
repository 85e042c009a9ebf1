"""C3-shaped decode timing (RS(255,223), 8 errors + 4 erasures per codeword, 1M codewords): the
decode call alone (HIP events around each call, the batch restored from a master copy before it),
with a check that the batch is restored.  Everything is generated on the device.  The library is
the default one or EZRS_LIB_VARIANT's.  Usage: c3_decode_time.py [reps]"""
import os, sys, time
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "ezpwd-reed-solomon_amd"))
import ezrs

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
ncw, n, k = 1 << 20, 255, 223
c = ezrs.Codec.rs(n, k)
c.reserve(ncw)
gen = torch.Generator(device="cuda").manual_seed(3)
clean = torch.randint(0, 256, (ncw, n), generator=gen, device="cuda", dtype=torch.int32).to(torch.uint8)
c.encode(clean, k)
units = [s for s in range(1, 40) if s % 3 and s % 5 and s % 17]
cop = torch.tensor(units, device="cuda")
b0 = torch.randint(0, n, (ncw, 1), generator=gen, device="cuda")
st = cop[torch.randint(0, len(units), (ncw, 1), generator=gen, device="cuda")]
locs = (b0 + torch.arange(12, device="cuda")[None, :] * st) % n          # 12 distinct positions
vals = torch.randint(1, 256, (ncw, 12), generator=gen, device="cuda", dtype=torch.int32).to(torch.uint8)
master = clean.clone()
master.scatter_(1, locs, master.gather(1, locs) ^ vals)
eras = torch.zeros((ncw, 32), dtype=torch.int32, device="cuda")
eras[:, :4] = locs[:, 8:].to(torch.int32)
neras = torch.full((ncw,), 4, dtype=torch.int32, device="cuda")
work = torch.empty_like(master)
result = torch.empty(ncw, dtype=torch.int32, device="cuda")
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
t0 = time.time()
while time.time() - t0 < 0.5:                   # clocks up
    for _ in range(5):
        work.copy_(master)
        c.decode(work, k, eras=eras, neras=neras, result=result)
    torch.cuda.synchronize()
for e0, e1 in evs:
    work.copy_(master)
    e0.record()
    c.decode(work, k, eras=eras, neras=neras, result=result)
    e1.record()
torch.cuda.synchronize()
ts = sorted(e0.elapsed_time(e1) for e0, e1 in evs)
ok = bool((result == 12).all()) and torch.equal(work, clean)
print(f"decode_ms={sum(ts) / len(ts):.4f} med={ts[len(ts) // 2]:.4f} min={ts[0]:.4f} ok={ok} "
      f"variant={os.path.basename(os.environ.get('EZRS_LIB_VARIANT', 'default'))}")
