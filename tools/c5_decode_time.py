"""C5-shaped timing (BCH(1023,983,4), 0-4 distinct bit errors per codeword): encode and decode calls
(HIP events around each, the batch restored from a master copy before each decode), with a check
that the batch is restored.  The library is the default one or EZRS_LIB_VARIANT's.
Usage: c5_decode_time.py [ncw] [reps]"""
import os, sys, time
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "ezpwd-reed-solomon_amd"))
import ezrs

ncw = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
L, row = 122, 127
c = ezrs.BCH.nkt(1023, 983, 4)
gen = torch.Generator(device="cuda").manual_seed(5)
clean = torch.randint(0, 256, (ncw, row), generator=gen, device="cuda", dtype=torch.int32).to(torch.uint8)
c.encode(clean, L)
nbits = 8 * L + 40
counts = torch.randint(0, 5, (ncw,), generator=gen, device="cuda", dtype=torch.int32)
pos = (torch.sort(torch.rand((ncw, 4), generator=gen, device="cuda"), dim=1).values
       * (nbits - 3)).to(torch.int64) + torch.arange(4, device="cuda")
master = clean.clone()
flat = master.view(-1)
for j in range(4):
    r = torch.nonzero(counts > j).squeeze(1)
    p = pos[r, j]
    idx = r * row + p // 8
    flat[idx] = flat[idx] ^ (128 >> (p % 8)).to(torch.uint8)
work = torch.empty_like(master)
res = torch.empty(ncw, dtype=torch.int32, device="cuda")
t0 = time.time()
while time.time() - t0 < 0.5:
    for _ in range(5):
        work.copy_(master)
        c.decode(work, L, result=res)
    torch.cuda.synchronize()
ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(reps)]
for e in ev:
    work.copy_(master)
    e[0].record()
    c.encode(clean, L)
    e[1].record()
    c.decode(work, L, result=res)
    e[2].record()
torch.cuda.synchronize()
enc = sum(e[0].elapsed_time(e[1]) for e in ev) / reps
dec = sum(e[1].elapsed_time(e[2]) for e in ev) / reps
ok = torch.equal(res, counts) and torch.equal(work, clean)
print(f"ncw={ncw} encode_ms={enc:.4f} decode_ms={dec:.4f} ok={ok} "
      f"variant={os.path.basename(os.environ.get('EZRS_LIB_VARIANT', 'default'))}")
