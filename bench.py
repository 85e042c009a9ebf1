#!/usr/bin/env python3
"""Headline benchmark: RS(255,223) encode+decode, device-resident, 1/2/4/8 MI355X.

BASELINE.json metric "RS(255,223) encode+decode GB/s device-resident", config C2 (configs[1]):
1,048,576 RS(255,223) codewords per GPU.  One step = encode every codeword of the batch (223 data
symbols -> 32 parity symbols, written into the codeword) followed by the errors-and-erasures decode
of every codeword (syndromes -> result; the batch is clean, as in C2).  value = codeword bytes
(255 B per codeword, the reference's exercise.H:248-267 unit) encoded AND decoded per second,
summed over all ranks.  Data starts and stays resident in HBM.

Multi-GPU: one process per GPU (torchrun), each rank owns its own 1M-codeword shard -- the path is
embarrassingly parallel, so there is no data-path collective (weak scaling); a barrier brackets the
timed region and the max time over ranks is taken.

Extra objects on the JSON line: "roofline" (dominant API call, algorithmic bytes / HIP-event
time vs 8 TB/s HBM), "cpu_baseline" (rank 0, N=1: the reference codec compiled from
/root/reference -- or the oracle restatement -- on the host cores, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "ezpwd-reed-solomon_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
N, K = 255, 223
NR = N - K
ENC_BYTES = K + NR              # per codeword: 223 B read + 32 B written
DEC_BYTES = N + 4               # per codeword: 255 B read + 4 B result written


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(seconds=12.0, threads=None):
    """Time the reference codec (oracle/_ref, compiled from /root/reference) -- or, if that build
    is absent, the oracle restatement -- on this host: RS(255,223) encode + clean decode of a
    bounded sample of the C2 workload, one slice per thread.  Returns the JSON object."""
    import numpy as np
    import oracle as O
    threads = threads or min(16, os.cpu_count() or 1)
    use_ref = O.Ref.available()
    if use_ref:
        idx = O.Ref.index("RS(255,223)")
        kind = "reference"
    else:
        oc = O.Codec(*O.rs_params(N, K))
        kind = "port"
    rng = np.random.default_rng(0x5EED0002)
    per = 4096
    bufs = [rng.integers(0, 256, (per, N)).astype(np.uint8) for _ in range(threads)]
    pars = [np.zeros((per, NR), np.uint8) for _ in range(threads)]

    def one(t):
        b, p = bufs[t], pars[t]
        if use_ref:
            O.Ref.encode_batch(idx, b, K, p)
            b[:, K:] = p
            O.Ref.decode_batch(idx, b, K, b[:, K:].copy())
        else:
            oc.encode_batch(b, K, None)
            oc.decode_batch(b, K, None)

    # calibrate on one round, then run enough rounds for ~`seconds` of wall time
    t0 = time.perf_counter()
    one(0)
    per_round = time.perf_counter() - t0
    rounds = max(1, int(seconds / max(per_round, 1e-6)))
    counts = [0] * threads

    def worker(t):
        for _ in range(rounds):
            one(t)
            counts[t] += per

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    ncw = sum(counts)
    return {"value": round(ncw * N / dt / 1e9, 4), "unit": "GB/s", "cores": threads,
            "kind": kind,
            "sample": f"RS(255,223) encode+clean decode of {ncw} random codewords "
                      f"({threads} threads x {rounds} rounds x {per} cw, {dt:.1f} s), "
                      f"{'reference ezpwd::RS<255,223> (oracle/_ref)' if use_ref else 'oracle restatement'}"}


def load_traffic(kernel_call):
    """HBM bytes per launch from the committed PMC summary (profiles/traffic.json), if any."""
    fn = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(fn) as f:
            t = json.load(f)
        return t.get(kernel_call, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def bench_rs_errors(args):
    """C3: RS(255,223), 1M codewords, each with 12 corrupted symbols of which the last 4 are passed as
    erasures (exercise.H:174-177); C4: RS(65535,65503), 65536 codewords (the full config; --ncw for
    fewer), same corruption.  One step = encode the clean batch + decode a corrupted copy (restored
    from a master before each decode, outside the timed kernels).  value = codeword bytes encoded
    and decoded per second of kernel time (HIP events), summed over ranks."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import ezrs
    import shard
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    c3 = args.workload == "c3"
    n, k = (255, 223) if c3 else (65535, 65503)
    ncw = args.ncw if (c3 or args.ncw != 1 << 20) else 65536     # C4: 64k codewords (configs[3])
    c = ezrs.Codec.rs(n, k, device=local)
    c.reserve(ncw)
    w = 1 if c3 else 2
    rng = np.random.default_rng(0x5EED0003 + rank)
    host = rng.integers(0, n + 1, (ncw, n)).astype(np.uint8 if c3 else np.uint16)
    tdt = torch.uint8 if c3 else torch.int16
    clean = torch.from_numpy(host.view(np.int16) if not c3 else host).cuda()
    if not c3:
        clean = clean.view(torch.uint16)
    c.encode(clean, k)
    torch.cuda.synchronize()
    enc = clean.view(tdt).cpu().numpy().view(host.dtype)
    bad = enc.copy()
    eras = np.zeros((ncw, 32), np.uint32)
    rows = np.arange(ncw)[:, None]
    locs = np.argsort(rng.random((ncw, n)), axis=1)[:, :12] if c3 else \
        np.stack([rng.choice(n, 12, replace=False) for _ in range(ncw)])
    bad[rows, locs] ^= rng.integers(1, n + 1, (ncw, 12)).astype(host.dtype)
    eras[:, :4] = locs[:, 8:]
    master = torch.from_numpy(bad.view(np.int16) if not c3 else bad).cuda()
    work = torch.empty_like(master)
    d_eras = torch.from_numpy(eras.view(np.int32)).cuda()
    d_neras = torch.full((ncw,), 4, dtype=torch.int32, device="cuda")
    result = torch.empty(ncw, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()

    def view(t):
        return t if c3 else t.view(torch.uint16)

    def step(ev=None):
        work.copy_(master)
        if ev:
            ev[0].record(stream)
        c.encode(view(clean), k, stream=stream)
        if ev:
            ev[1].record(stream)
        c.decode(view(work), k, eras=d_eras, neras=d_neras, result=result, stream=stream)
        if ev:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if not bool((result == 12).all()) or not torch.equal(work, clean.view(work.dtype)):
        raise SystemExit(f"rank {rank}: {args.workload} decode did not restore the batch")
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    for s_ in range(args.steps):
        step(evs[s_])
    torch.cuda.synchronize()
    enc_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    dec_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
    t = shard.max_over_ranks(enc_ms + dec_ms, device="cuda")
    row = n * w
    value = ncw * world * row / (t * 1e-3) / 1e9
    dom, ms, per = ("ezrs_encode", enc_ms, row) if enc_ms >= dec_ms else ("ezrs_decode", dec_ms, row + 4)
    achieved = ncw * per / (ms * 1e-3) / 1e9
    if rank == 0:
        print(json.dumps({
            "metric": f"RS({n},{k}) encode + 8-error/4-erasure decode GB/s device-resident "
                      f"({args.workload.upper()})",
            "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8" if c3 else "u16",
            "data": "synthetic",
            "config": {"workload": f"{args.workload.upper()}: RS({n},{k}) encode + decode of 8 errors "
                                   f"+ 4 erasures per codeword (restore copy excluded)",
                       "codewords_per_gpu": ncw, "bytes_per_codeword": row,
                       "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None, "kernel": dom,
                         "avg_ms": {"ezrs_encode": round(enc_ms, 4), "ezrs_decode": round(dec_ms, 4)}},
            "cpu_baseline": None}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_c5(args):
    """C5: BCH(1023,983,4), 1M codewords of 122 data + 5 ECC bytes per GPU.  One step = encode the
    clean batch + decode a batch carrying 0..4 random bit errors per codeword (restored from a
    corrupted master copy before each decode; that copy is outside the timed kernels).  value =
    codeword bytes encoded and decoded per second of kernel time (HIP events), summed over ranks."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import ezrs
    import shard
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    c = ezrs.BCH.nkt(1023, 983, 4, device=local)
    ncw, L, row = args.ncw, 122, 127
    gen = torch.Generator(device="cuda").manual_seed(0x5EED0005 + rank)
    clean = torch.randint(0, 256, (ncw, row), generator=gen, device="cuda", dtype=torch.int32)
    clean = clean.to(torch.uint8)
    c.encode(clean, L)
    rng = np.random.default_rng(5 + rank)
    nbits = 8 * L + 40
    counts = rng.integers(0, 5, ncw)
    pos = (np.sort(rng.random((ncw, 4)), axis=1) * (nbits - 3)).astype(np.int64) + np.arange(4)
    bad = clean.cpu().numpy()
    for j in range(4):
        r = np.nonzero(counts > j)[0]
        p = pos[r, j]
        bad[r, p // 8] ^= (0x80 >> (p % 8)).astype(np.uint8)
    master = torch.from_numpy(bad).cuda()
    work = torch.empty_like(master)
    result = torch.empty(ncw, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()
    exp = torch.from_numpy(counts.astype(np.int32)).cuda()

    def step(ev=None):
        work.copy_(master)
        if ev:
            ev[0].record(stream)
        c.encode(clean, L, stream=stream)
        if ev:
            ev[1].record(stream)
        c.decode(work, L, result=result, stream=stream)
        if ev:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if not torch.equal(result, exp) or not torch.equal(work, clean):
        raise SystemExit(f"rank {rank}: C5 decode did not restore the batch")
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    for s in range(args.steps):
        step(evs[s])
    torch.cuda.synchronize()
    enc_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    dec_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
    t = shard.max_over_ranks(enc_ms + dec_ms, device="cuda")
    value = ncw * world * row / (t * 1e-3) / 1e9
    dom, ms, per = ("ezbch_encode", enc_ms, row) if enc_ms >= dec_ms else ("ezbch_decode", dec_ms, row + 4)
    achieved = ncw * per / (ms * 1e-3) / 1e9
    if rank == 0:
        print(json.dumps({
            "metric": "BCH(1023,983,4) encode+decode GB/s device-resident (C5)",
            "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": "C5: BCH(1023,983,4) encode + decode with 0-4 bit errors, "
                                   "1M codewords/GPU (restore copy excluded)",
                       "codewords_per_gpu": ncw, "bytes_per_codeword": row,
                       "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic(dom), "kernel": dom,
                         "avg_ms": {"ezbch_encode": round(enc_ms, 4),
                                    "ezbch_decode": round(dec_ms, 4)}},
            "cpu_baseline": None}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--ncw", type=int, default=1 << 20, help="codewords per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--e2e", action="store_true", help="also time the host-memory pipeline")
    ap.add_argument("--workload", choices=("c2", "c3", "c4", "c5"), default="c2",
                    help="c2: the headline RS(255,223) line; c3: RS(255,223) 8 errors + 4 erasures "
                         "decode; c4: RS(65535,65503); c5: BCH(1023,983,4) (SURVEY.md 8d)")
    args = ap.parse_args()
    if args.workload == "c5":
        return bench_c5(args)
    if args.workload in ("c3", "c4"):
        return bench_rs_errors(args)

    import torch
    import torch.distributed as dist
    import ezrs
    import shard

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    codec = ezrs.Codec.rs(N, K, device=local)
    ncw = args.ncw
    codec.reserve(ncw)
    gen = torch.Generator(device="cuda").manual_seed(0x5EED0002 + rank)
    cw = torch.randint(0, 256, (ncw, N), generator=gen, device="cuda", dtype=torch.int32)
    cw = cw.to(torch.uint8)
    result = torch.empty(ncw, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()

    def step(ev=None):
        if ev:
            ev[0].record(stream)
        codec.encode(cw, K, stream=stream)
        if ev:
            ev[1].record(stream)
        codec.decode(cw, K, result=result, stream=stream)
        if ev:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    bad = int((result != 0).sum())
    if bad:
        raise SystemExit(f"rank {rank}: {bad} encoded codewords did not decode clean")

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        step(evs[s])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    enc_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    dec_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
    elapsed = shard.max_over_ranks(elapsed, device="cuda")

    total_cw = ncw * world * args.steps
    value = total_cw * N / elapsed / 1e9
    if enc_ms >= dec_ms:
        dom, ms, per_cw = "ezrs_encode", enc_ms, ENC_BYTES
    else:
        dom, ms, per_cw = "ezrs_decode", dec_ms, DEC_BYTES
    achieved = ncw * per_cw / (ms * 1e-3) / 1e9
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": load_traffic(dom), "kernel": dom,
                "algorithmic_bytes_per_launch": ncw * per_cw,
                "avg_ms": {"ezrs_encode": round(enc_ms, 4), "ezrs_decode": round(dec_ms, 4)}}

    e2e = None
    if args.e2e and rank == 0:
        import numpy as np
        h = np.random.default_rng(3).integers(0, 256, (ncw, N)).astype(np.uint8)
        # pinned (page-locked, hipHostMalloc via torch) copy of the same batch: the north_star's
        # "pinned hipMemcpyAsync" end-to-end rate; the pageable numpy rate is reported beside it
        hp = torch.from_numpy(h.copy()).pin_memory().numpy()
        e2e = {}
        for name, buf in (("pageable", h), ("pinned", hp)):
            codec.encode_host(buf, K)
            t1 = time.perf_counter()
            for _ in range(3):
                codec.encode_host(buf, K)
                r = codec.decode_host(buf, K)
            dt = (time.perf_counter() - t1) / 3
            assert (r == 0).all()
            e2e[name] = round(ncw * N / dt / 1e9, 3)
            log(f"host-memory ({name}) encode+decode: {e2e[name]} GB/s")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds)

    if rank == 0:
        line = {"metric": "RS(255,223) encode+decode GB/s device-resident",
                "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": "u8", "data": "synthetic",
                "config": {"workload": "C2: RS(255,223) encode + clean decode, 1M codewords/GPU",
                           "codec": "RS(255,223) poly 0x11d fcr 1 prim 1",
                           "codewords_per_gpu": ncw, "global_codewords": ncw * world,
                           "bytes_per_codeword": N, "parallelism": f"shard{world}"},
                "roofline": roofline, "cpu_baseline": cpu}
        if e2e is not None:
            line["e2e_host_gbs"] = e2e
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
