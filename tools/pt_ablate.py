#!/usr/bin/env python3
"""Timing-only ablations of the tile kernel (EZRS_PT_ABLATE bits, see PsArgs::ablate): per variant,
the device time of ezrs_encode and ezrs_decode on 1M RS(255,223) rows.  Results are garbage
under ablation; nothing is checked.  Needs a variant library built with the env hook:
  tools/build_variant.sh ablate -DEZRS_PT_ABLATE_ENV, then EZRS_LIB_VARIANT=<path>.
Usage: python tools/pt_ablate.py [bits ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ezpwd-reed-solomon_amd"))
import torch  # noqa: E402
import ezrs  # noqa: E402

ncw = 1 << 20
c = ezrs.Codec.rs(255, 223)
c.reserve(ncw)
cw = torch.randint(0, 256, (ncw, 255), device="cuda", dtype=torch.int32).to(torch.uint8)
res = torch.empty(ncw, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
for bits in (sys.argv[1:] or ["0"]):
    os.environ["EZRS_PT_ABLATE"] = str(int(bits) | 32)
    for _ in range(3):
        c.encode(cw, 223, stream=s)
        c.decode(cw, 223, result=res, stream=s)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    te = td = 0.0
    n = 20
    for _ in range(n):
        ev[0].record(s)
        c.encode(cw, 223, stream=s)
        ev[1].record(s)
        c.decode(cw, 223, result=res, stream=s)
        ev[2].record(s)
        torch.cuda.synchronize()
        te += ev[0].elapsed_time(ev[1])
        td += ev[1].elapsed_time(ev[2])
    print(f"ablate={bits:>3}  encode {1e3 * te / n:8.1f} us  decode {1e3 * td / n:8.1f} us", flush=True)
