#!/usr/bin/env python3
"""Per-step GPU timing of the C2 step (encode + clean decode of 1M RS(255,223) codewords) right
after a host synchronize: does a timed region that starts from an idle GPU pay a ramp, and how long?

Prints, for each mode, the first 12 per-step times (HIP events, one pair per step) and the mean of
the rest.  Modes: 'sync' (warm-up, synchronize, then the steps: the bench contract), 'nosync'
(warm-up immediately followed by the steps on the same stream).  Timing experiment only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ezpwd-reed-solomon_amd"))

import torch  # noqa: E402
import ezrs  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    c = ezrs.Codec.rs(255, 223, device=0)
    ncw = 1 << 20
    c.reserve(ncw)
    g = torch.Generator(device="cuda").manual_seed(1)
    cw = torch.randint(0, 256, (ncw, 255), generator=g, device="cuda", dtype=torch.int32).to(torch.uint8)
    res = torch.empty(ncw, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()

    def step():
        c.encode(cw, 223, stream=st)
        c.decode(cw, 223, result=res, stream=st)

    for mode in ("sync", "nosync", "sync", "idle10ms"):
        for _ in range(20):
            step()
        if mode in ("sync", "idle10ms"):
            torch.cuda.synchronize()
        if mode == "idle10ms":
            time.sleep(0.01)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        t0 = time.perf_counter()
        ev[0].record(st)
        for i in range(steps):
            step()
            ev[i + 1].record(st)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        d = [ev[i].elapsed_time(ev[i + 1]) for i in range(steps)]
        print(f"{mode:9s} wall {wall:7.3f} ms  events {sum(d):7.3f} ms  first12 "
              + " ".join(f"{x:.3f}" for x in d[:12]) + f"  rest-mean {sum(d[12:]) / max(1, steps - 12):.4f}",
              flush=True)


if __name__ == "__main__":
    main()
