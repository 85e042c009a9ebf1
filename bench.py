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


SHARE_GPUS = False              # --share-gpus: ranks may share a GPU (harness test only)


def bench_device(local):
    """This rank's GPU: LOCAL_RANK, one GPU per rank.  More ranks than visible GPUs is an error
    unless --share-gpus was given (tests/test_bench_gpu.py runs --gpus 2 on a one-GPU box): then
    ranks wrap around the devices and the JSON line says so (gpu_fields).  The process group is gloo
    on CPU: the only cross-rank traffic is the barrier and the scalar max/sum of the timing rule, so
    no RCCL communicator is ever needed."""
    import torch
    ndev = max(1, torch.cuda.device_count())
    if local >= ndev and not SHARE_GPUS:
        raise SystemExit(f"bench: LOCAL_RANK {local} but only {ndev} visible GPU(s); one rank per "
                         "GPU is required (--share-gpus lets ranks share GPUs, never a scaling run)")
    dev = local % ndev
    torch.cuda.set_device(dev)
    return dev


def gpu_fields(world):
    """n_gpus / scaling of the JSON line: the distinct devices the ranks ran on.  A run whose ranks
    share GPUs (--share-gpus) is marked so that it is never read as a scaling measurement."""
    import torch
    ndev = max(1, torch.cuda.device_count())
    if world <= ndev:
        return {"n_gpus": world, "scaling": "weak"}
    return {"n_gpus": ndev, "ranks": world, "shared_gpus": True,
            "scaling": "none (ranks share GPUs: harness check, not a scaling measurement)"}


def host_cpu_info():
    """CPU model, logical CPUs (nproc), the CPUs this process may run on, the cgroup CPU quota
    and the physical core count of the host."""
    info = {"model": "?", "nproc": os.cpu_count() or 1}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = info["nproc"]
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    info["cgroup_quota"] = quota
    try:
        import subprocess
        out = subprocess.run(["lscpu", "-p=core,socket"], capture_output=True, text=True,
                             timeout=10).stdout
        cores = {tuple(l.split(",")[:2]) for l in out.splitlines() if l and not l.startswith("#")}
        info["physical_cores"] = len(cores) or None
    except Exception:
        info["physical_cores"] = None
    usable = min(x for x in (info["affinity"], quota, info["physical_cores"]) if x)
    info["threads_used"] = usable
    return info


def _time_threads(one, threads, seconds):
    """Run one(t) repeatedly on `threads` threads for about `seconds`; returns (items, dt)."""
    t0 = time.perf_counter()
    n0 = one(0)
    per_round = time.perf_counter() - t0
    rounds = max(1, int(seconds / max(per_round, 1e-6)))
    counts = [0] * threads

    def worker(t):
        for _ in range(rounds):
            counts[t] += one(t)

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    return sum(counts), time.perf_counter() - t0


def cpu_baselines(seconds=4.0):
    """The reference codec (oracle/_ref, compiled from /root/reference; the oracle restatement
    where that build or codec is absent) timed on this host's cores, single-threaded and on every
    usable physical core, for the SURVEY 8(d) configs: C2 (the headline), C1, C3, C4 and C5 (BCH:
    the restatement of the absent Djelic library).  Bounded samples of `seconds` each.  Returns the
    cpu_baseline object of the C2 line (value = all-core C2 rate) with the other rows attached."""
    import numpy as np
    import oracle as O
    info = host_cpu_info()
    nth = info["threads_used"]
    use_ref = O.Ref.available()
    rng = np.random.default_rng(0x5EED0002)

    def rs_rows(n, k, per, nerr, nera, dtype=np.uint8):
        """`per` encoded rows + corrupted copies (nerr errors + nera erasures per row)."""
        nn = n if dtype == np.uint8 else 65535
        data = rng.integers(0, nn + 1, (per, n)).astype(dtype)
        oc = O.Codec(*O.rs_params(n, k))
        oc.encode_batch(data, k, None, nthreads=8)
        bad = data.copy()
        eras = np.zeros((per, max(1, n - k)), np.uint32)
        neras = np.zeros(per, np.uint32)
        if nerr + nera:
            for r in range(per):
                locs = rng.choice(n, nerr + nera, replace=False)
                bad[r, locs] ^= rng.integers(1, nn + 1, nerr + nera).astype(dtype)
                eras[r, :nera] = locs[nerr:]
            neras[:] = nera
        return data, bad, eras, neras

    def rs_case(name, n, k, per, nerr, nera, encode, dtype=np.uint8):
        data, bad, eras, neras = rs_rows(n, k, per, nerr, nera, dtype)
        idx = None
        if use_ref:
            try:
                idx = O.Ref.index(f"RS({n},{k})")
            except KeyError:
                idx = None
        oc = O.Codec(*O.rs_params(n, k))
        bufs = {}

        def one(t):
            if t not in bufs:
                bufs[t] = (data.copy(), bad.copy(), np.zeros((per, n - k), dtype))
            d, b, p = bufs[t]
            if nerr + nera:
                b[:] = bad                    # corrections are in place: restore the input
            if idx is not None:
                L = O.Ref.lib()
                if encode:
                    L.ezref_encode_batch(idx, d.ctypes.data, n, k,
                                         p.ctypes.data, n - k, per, d.itemsize)
                # inline parity: the parity of row r starts at b[r, k] (stride n)
                L.ezref_decode_batch(idx, b.ctypes.data, n, k, b.ctypes.data + k * b.itemsize, n,
                                     eras.ctypes.data if nera else None, eras.shape[1],
                                     neras.ctypes.data if nera else None, res.ctypes.data, None, 0,
                                     per, b.itemsize)
            else:
                if encode:
                    oc.encode_batch(d, k, p)
                oc.decode_batch(b, k, None, eras if nera else None, neras if nera else None)
            return per
        res = np.zeros(per, np.int32)
        row = {"workload": name, "kind": "reference" if idx is not None else "port"}
        for label, th in (("threads_1", 1), ("threads_all", nth)):
            ncw, dt = _time_threads(one, th, seconds)
            row[label] = round(ncw * n * np.dtype(dtype).itemsize / dt / 1e9, 5)
            row[label + "_sample"] = f"{ncw} codewords in {dt:.2f} s"
        return row

    rows = {
        "C2": rs_case("RS(255,223) encode + clean decode", 255, 223, 4096, 0, 0, True),
        "C1": rs_case("RS(255,251) encode + decode, 1 error per codeword", 255, 251, 10000, 1, 0,
                      True),
        "C3": rs_case("RS(255,223) decode, 8 errors + 4 erasures", 255, 223, 2048, 8, 4, False),
        "C4": rs_case("RS(65535,65503) encode + decode, 8 errors + 4 erasures", 65535, 65503, 16,
                      8, 4, True, np.uint16),
    }
    # C5: BCH(1023,983,4), 122 data + 5 ECC bytes, 0..4 bit errors (restatement: Djelic is absent)
    b = O.BCH(10, 4)
    per = 20000
    d = rng.integers(0, 256, (per, 127)).astype(np.uint8)
    b.encode_batch(d, 122, None, nthreads=8)
    bad = d.copy()
    cnt = rng.integers(0, 5, per)
    for r in range(per):
        for p in rng.choice(8 * 127, int(cnt[r]), replace=False):
            bad[r, p // 8] ^= np.uint8(0x80 >> (p % 8))
    bb = {}

    def one5(t):
        if t not in bb:
            bb[t] = (d.copy(), bad.copy())
        x, y = bb[t]
        b.encode_batch(x, 122, None)
        y[:] = bad
        b.decode_batch(y, 122, None)
        return per
    c5 = {"workload": "BCH(1023,983,4) encode + decode, 0-4 bit errors", "kind": "port"}
    for label, th in (("threads_1", 1), ("threads_all", nth)):
        ncw, dt = _time_threads(one5, th, seconds)
        c5[label] = round(ncw * 127 / dt / 1e9, 5)
        c5[label + "_sample"] = f"{ncw} codewords in {dt:.2f} s"
    rows["C5"] = c5
    c2 = rows["C2"]
    return {"value": c2["threads_all"], "unit": "GB/s", "cores": nth, "kind": c2["kind"],
            "sample": f"RS(255,223) encode+clean decode, {c2['threads_all_sample']} on {nth} "
                      f"threads ({'reference ezpwd::RS<255,223>, oracle/_ref' if c2['kind'] == 'reference' else 'oracle restatement'})",
            "single_thread": c2["threads_1"], "cpu_model": info["model"], "nproc": info["nproc"],
            "affinity_cpus": info["affinity"], "cgroup_quota": info["cgroup_quota"],
            "physical_cores": info["physical_cores"], "rows": rows}


def load_traffic(workload, kernel_call, ncw):
    """HBM bytes per launch of `kernel_call` in `workload` from the committed PMC summary
    (profiles/traffic.json, tools/traffic_json.py), when it was measured at this batch size."""
    fn = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(fn) as f:
            t = json.load(f).get(workload, {})
        if t.get("codewords") != ncw:
            return None
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
    local = bench_device(local)
    if world > 1:
        dist.init_process_group("gloo")
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
    t = shard.max_over_ranks(enc_ms + dec_ms)
    row = n * w
    value = ncw * world * row / (t * 1e-3) / 1e9
    dom, ms, per = ("ezrs_encode", enc_ms, row) if enc_ms >= dec_ms else ("ezrs_decode", dec_ms, row + 4)
    achieved = ncw * per / (ms * 1e-3) / 1e9
    if rank == 0:
        print(json.dumps({
            "metric": f"RS({n},{k}) encode + 8-error/4-erasure decode GB/s device-resident "
                      f"({args.workload.upper()})",
            "value": round(value, 3), "unit": "GB/s", **gpu_fields(world), "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t, 4), "higher_is_better": True,
            "vs_baseline": None, "dtype": "u8" if c3 else "u16",
            "data": "synthetic",
            "config": {"workload": f"{args.workload.upper()}: RS({n},{k}) encode + decode of 8 errors "
                                   f"+ 4 erasures per codeword (restore copy excluded)",
                       "codewords_per_gpu": ncw, "bytes_per_codeword": row,
                       "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic(args.workload, dom, ncw), "kernel": dom,
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
    local = bench_device(local)
    if world > 1:
        dist.init_process_group("gloo")
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
    t = shard.max_over_ranks(enc_ms + dec_ms)
    value = ncw * world * row / (t * 1e-3) / 1e9
    dom, ms, per = ("ezbch_encode", enc_ms, row) if enc_ms >= dec_ms else ("ezbch_decode", dec_ms, row + 4)
    achieved = ncw * per / (ms * 1e-3) / 1e9
    if rank == 0:
        print(json.dumps({
            "metric": "BCH(1023,983,4) encode+decode GB/s device-resident (C5)",
            "value": round(value, 3), "unit": "GB/s", **gpu_fields(world), "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t, 4), "higher_is_better": True,
            "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": "C5: BCH(1023,983,4) encode + decode with 0-4 bit errors, "
                                   f"{ncw} codewords/GPU (restore copy excluded)",
                       "codewords_per_gpu": ncw, "bytes_per_codeword": row,
                       "parallelism": f"shard{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic("c5", dom, ncw), "kernel": dom,
                         "avg_ms": {"ezbch_encode": round(enc_ms, 4),
                                    "ezbch_decode": round(dec_ms, 4)}},
            "cpu_baseline": None}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def relaunch_distributed(args):
    """`bench.py --gpus N` started directly (not under torchrun): run N ranks, one process per GPU,
    through torch.distributed.run on this node, and return its exit status.  Nothing here touches
    the GPU before the ranks are started."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", "--master-port",
           str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    log(f"bench: launching {args.gpus} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd, env=env)


def harness_check(args):
    """The multi-rank harness alone, on CPU with gloo (tests/test_bench_harness.py): the same
    launch, barrier + max-over-ranks timing and JSON line as the GPU workloads, with a placeholder
    step (an XOR pass over a host buffer, no codec work).  Never a measurement."""
    import numpy as np
    import torch.distributed as dist
    import shard
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("gloo")
    lo, hi = shard.shard_range(args.ncw * world, world, rank)
    buf = np.random.default_rng(rank).integers(0, 256, (hi - lo, 255), dtype=np.uint8)
    acc = np.zeros(255, np.uint8)
    for _ in range(args.warmup):
        np.bitwise_xor.reduce(buf, axis=0, out=acc)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        np.bitwise_xor.reduce(buf, axis=0, out=acc)
    if world > 1:
        dist.barrier()
    t = shard.max_over_ranks(time.perf_counter() - t0)
    counts = shard.sum_over_ranks([hi - lo])
    if rank == 0:
        print(json.dumps({"metric": "harness check (no codec work)", "value": None, "unit": None,
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(t / args.steps * 1e3, 4),
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                          "dtype": "u8", "data": "harness check: placeholder step, gloo, CPU",
                          "config": {"workload": "harness", "codewords_total": counts[0],
                                     "parallelism": f"shard{world}"},
                          "roofline": None, "cpu_baseline": None}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def shard_point(codec, S, steps, warmup, gen):
    """One shard size of the sweep: ~256 MB of S-byte shards, encode_shards + decode_shards timed
    with HIP events (one launch each), the rates and HBM fractions of both calls."""
    import torch
    shards = max(1, (256 << 20) // S)
    R = codec.shard_codewords(S)
    enc = codec.shard_encoded_len(S)
    buf = torch.randint(0, 256, (shards, enc), generator=gen, device="cuda",
                        dtype=torch.int32).to(torch.uint8)
    codec.reserve(shards * R)
    res = torch.empty(shards * R, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()

    def step(ev=None):
        if ev:
            ev[0].record(stream)
        codec.encode_shards(buf, S, stream=stream)
        if ev:
            ev[1].record(stream)
        codec.decode_shards(buf, S, result=res, stream=stream)
        if ev:
            ev[2].record(stream)
    for _ in range(max(1, warmup)):
        step()
    torch.cuda.synchronize()
    if int((res != 0).sum()):
        raise SystemExit(f"shards S={S}: encoded shards did not decode clean")
    steps = max(1, steps)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    t0 = time.perf_counter()
    for i in range(steps):
        step(evs[i])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    enc_ms = sum(e[0].elapsed_time(e[1]) for e in evs) / steps
    dec_ms = sum(e[1].elapsed_time(e[2]) for e in evs) / steps
    enc_alg = shards * enc                         # data read + parity written
    dec_alg = enc_alg + 4 * shards * R             # all read + result written
    return {"shard_bytes": S, "shards": shards, "codewords": shards * R,
            "tail_len": S - (R - 1) * K, "gbs_shard_data": round(shards * S / dt / 1e9, 3),
            "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
            "frac_encode": round(enc_alg / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "frac_decode": round(dec_alg / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}


def timed_pair(enc_fn, dec_fn, steps, warmup, pre=None):
    """Average HIP-event time (ms) of enc_fn and dec_fn on the current stream over `steps` steps;
    pre() (outside the events) runs before each step.  The warm-up steps are enqueued right before
    the timed ones with no host synchronize in between, so the timed calls never start from an idle
    GPU (an idle gap costs the next ~2 ms a clock ramp: DESIGN.md 5)."""
    import torch
    stream = torch.cuda.current_stream()
    for _ in range(max(1, warmup)):
        if pre:
            pre()
        enc_fn(stream)
        dec_fn(stream)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    for e in evs:
        if pre:
            pre()
        e[0].record(stream)
        enc_fn(stream)
        e[1].record(stream)
        dec_fn(stream)
        e[2].record(stream)
    torch.cuda.synchronize()
    return (sum(e[0].elapsed_time(e[1]) for e in evs) / steps,
            sum(e[1].elapsed_time(e[2]) for e in evs) / steps)


def uniform_positions(gen, rows, n, m, rows_per_chunk=1 << 17):
    """[rows, m] int64: per row m distinct positions drawn uniformly from [0, n) (the indices of the
    m largest of n uniform draws: a uniformly random m-subset in random order), on the device."""
    import torch
    out = torch.empty((rows, m), dtype=torch.int64, device="cuda")
    for r0 in range(0, rows, rows_per_chunk):
        nr = min(rows_per_chunk, rows - r0)
        out[r0:r0 + nr] = torch.rand((nr, n), generator=gen, device="cuda").topk(m, dim=1).indices
    return out


def c4_extra(gen, steps=3):
    """SURVEY 8(d) C4 on the default line: RS(65535,65503), 65 536 codewords (8.6 GB of 16-bit
    symbols, BASELINE configs[3], rsexercise.C:27-28), each with 12 distinct corrupted symbols of
    which the last 4 are passed as erasures.  Everything is generated on the device."""
    import torch
    import ezrs
    n, k, ncw = 65535, 65503, 65536
    c = ezrs.Codec.rs(n, k, device=torch.cuda.current_device())
    c.reserve(ncw)
    clean = torch.empty((ncw, n), dtype=torch.int16, device="cuda")
    for r0 in range(0, ncw, 4096):
        clean[r0:r0 + 4096] = torch.randint(-32768, 32768, (min(4096, ncw - r0), n), generator=gen,
                                            device="cuda", dtype=torch.int16)
    u16 = clean.view(torch.uint16)
    c.encode(u16, k)
    locs = uniform_positions(gen, ncw, n, 12, rows_per_chunk=2048)   # distinct, uniform
    vals = torch.randint(1, 65536, (ncw, 12), generator=gen, device="cuda", dtype=torch.int32).to(torch.int16)
    master = clean.clone()
    master.scatter_(1, locs, master.gather(1, locs) ^ vals)
    eras = locs[:, 8:].to(torch.int32).contiguous()
    neras = torch.full((ncw,), 4, dtype=torch.int32, device="cuda")
    work = torch.empty_like(master)
    res = torch.empty(ncw, dtype=torch.int32, device="cuda")
    e_ms, d_ms = timed_pair(lambda s_: c.encode(u16, k, stream=s_),
                            lambda s_: c.decode(work.view(torch.uint16), k, eras=eras, neras=neras,
                                                result=res, stream=s_),
                            steps, 1, pre=lambda: work.copy_(master))
    if not bool((res == 12).all()) or not torch.equal(work, clean):
        raise SystemExit("C4 extra: decode did not restore the batch")
    row = 2 * n
    out = {"codewords": ncw, "encode_ms": round(e_ms, 4), "decode_ms": round(d_ms, 4),
           "value_gbs": round(ncw * row / ((e_ms + d_ms) * 1e-3) / 1e9, 3),
           "frac_encode": round(ncw * row / (e_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "frac_decode": round(ncw * (row + 4) / (d_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "traffic": {"ezrs_encode": load_traffic("c4", "ezrs_encode", ncw),
                       "ezrs_decode": load_traffic("c4", "ezrs_decode", ncw)}}
    del clean, master, work, res, u16
    torch.cuda.empty_cache()
    return out


def c5_extra(gen, steps=5, ncw=8 << 20):
    """SURVEY 8(d) C5 on the default line: BCH(1023,983,4), the config's full 8M-codeword batch on
    this one GPU (122 data + 5 ECC bytes, bch:196-205,316-331), decode inputs carrying 0..4 random
    bit errors per codeword (distinct bits).  Everything is generated on the device."""
    import torch
    import ezrs
    L, row = 122, 127
    c = ezrs.BCH.nkt(1023, 983, 4, device=torch.cuda.current_device())
    clean = torch.empty((ncw, row), dtype=torch.uint8, device="cuda")
    for r0 in range(0, ncw, 1 << 20):
        clean[r0:r0 + (1 << 20)] = torch.randint(0, 256, (min(1 << 20, ncw - r0), row), generator=gen,
                                                 device="cuda", dtype=torch.int32).to(torch.uint8)
    c.encode(clean, L)
    nbits = 8 * L + 40
    counts = torch.randint(0, 5, (ncw,), generator=gen, device="cuda", dtype=torch.int32)
    pos = (torch.sort(torch.rand((ncw, 4), generator=gen, device="cuda"), dim=1).values
           * (nbits - 3)).to(torch.int64) + torch.arange(4, device="cuda")       # distinct bits
    master = clean.clone()
    flat = master.view(-1)
    for j in range(4):
        r = torch.nonzero(counts > j).squeeze(1)
        p = pos[r, j]
        idx = r * row + p // 8
        flat[idx] = flat[idx] ^ (128 >> (p % 8)).to(torch.uint8)
    work = torch.empty_like(master)
    res = torch.empty(ncw, dtype=torch.int32, device="cuda")
    e_ms, d_ms = timed_pair(lambda s_: c.encode(clean, L, stream=s_),
                            lambda s_: c.decode(work, L, result=res, stream=s_),
                            steps, 3, pre=lambda: work.copy_(master))
    if not torch.equal(res, counts) or not torch.equal(work, clean):
        raise SystemExit("C5 extra: decode did not restore the batch")
    out = {"codewords": ncw, "encode_ms": round(e_ms, 4), "decode_ms": round(d_ms, 4),
           "value_gbs": round(ncw * row / ((e_ms + d_ms) * 1e-3) / 1e9, 3),
           "frac_encode": round(ncw * row / (e_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "frac_decode": round(ncw * (row + 4) / (d_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "traffic": {"ezbch_encode": load_traffic("c5_8m", "ezbch_encode", ncw),
                       "ezbch_decode": load_traffic("c5_8m", "ezbch_decode", ncw)}}
    del clean, master, work, res
    torch.cuda.empty_cache()
    return out


def c2_extras(codec, args):
    """The north_star / SURVEY 8(d) figures the driver's default run carries beside the headline
    (all timed in the same process, HIP events): shard batches at S = 1 KiB and 1 MiB, C2 at 4M
    codewords (1.07 GB, past the 256 MiB Infinity Cache), the C3 decode (8 errors + 4 erasures per
    codeword), C4 (RS(65535,65503), 64k codewords), C5 (BCH(1023,983,4), 8M codewords), and the
    host-memory (PCIe-inclusive) rates, clean and with 1 % of the rows corrupted.  None of these
    is `value`."""
    import numpy as np
    import torch
    out = {}
    gen = torch.Generator(device="cuda").manual_seed(0x5EED0007)
    out["shards"] = {}
    for S in (1 << 10, 1 << 20):
        r = shard_point(codec, S, max(3, args.steps // 2), 1, gen)
        out["shards"][f"{S // 1024}KiB"] = r
        log(f"extras: shards S={S}: {r}")
    torch.cuda.empty_cache()
    # C2 at 4M codewords
    n4 = 4 << 20
    big = torch.randint(0, 256, (n4, N), generator=gen, device="cuda", dtype=torch.int32).to(torch.uint8)
    codec.reserve(n4)
    res4 = torch.empty(n4, dtype=torch.int32, device="cuda")
    e_ms, d_ms = timed_pair(lambda st: codec.encode(big, K, stream=st),
                            lambda st: codec.decode(big, K, result=res4, stream=st), 5, 1)
    if int((res4 != 0).sum()):
        raise SystemExit("C2 4M: encoded codewords did not decode clean")
    out["c2_4m"] = {"codewords": n4, "encode_ms": round(e_ms, 4), "decode_ms": round(d_ms, 4),
                    "value_gbs": round(n4 * N / ((e_ms + d_ms) * 1e-3) / 1e9, 3),
                    "frac_encode": round(n4 * ENC_BYTES / (e_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "frac_decode": round(n4 * DEC_BYTES / (d_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    log(f"extras: c2_4m {out['c2_4m']}")
    del big, res4
    torch.cuda.empty_cache()
    # C3: 1M codewords, 12 distinct corrupted symbols at positions uniform over [0, 255) (SURVEY
    # 8(d)), the last 4 passed as erasures; the corrupted master is copied in before each step
    # (outside the events)
    ncw = 1 << 20
    clean = torch.randint(0, 256, (ncw, N), generator=gen, device="cuda", dtype=torch.int32).to(torch.uint8)
    codec.encode(clean, K)
    locs = uniform_positions(gen, ncw, N, 12)
    vals = torch.randint(1, 256, (ncw, 12), generator=gen, device="cuda", dtype=torch.int32).to(torch.uint8)
    master = clean.clone()
    master.scatter_(1, locs, master.gather(1, locs) ^ vals)
    eras = locs[:, 8:].to(torch.int32).contiguous()
    neras = torch.full((ncw,), 4, dtype=torch.int32, device="cuda")
    work = torch.empty_like(master)
    res = torch.empty(ncw, dtype=torch.int32, device="cuda")
    codec.reserve(ncw)
    e_ms, d_ms = timed_pair(lambda st: codec.encode(clean, K, stream=st),
                            lambda st: codec.decode(work, K, eras=eras, neras=neras, result=res, stream=st),
                            10, 8, pre=lambda: work.copy_(master))
    if not bool((res == 12).all()) or not torch.equal(work, clean):
        raise SystemExit("C3 extra: decode did not restore the batch")
    out["c3"] = {"codewords": ncw, "decode_ms": round(d_ms, 4), "encode_ms": round(e_ms, 4),
                 "frac_decode": round(ncw * DEC_BYTES / (d_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                 "traffic": {"ezrs_encode": load_traffic("c3", "ezrs_encode", ncw),
                             "ezrs_decode": load_traffic("c3", "ezrs_decode", ncw)}}
    log(f"extras: c3 {out['c3']}")
    del clean, master, work, res, locs, vals, eras, neras
    torch.cuda.empty_cache()
    out["c4"] = c4_extra(gen)
    log(f"extras: c4 {out['c4']}")
    out["c5"] = c5_extra(gen)
    log(f"extras: c5 {out['c5']}")
    # host-memory pipeline (the north_star's PCIe-inclusive rate)
    h = np.random.default_rng(3).integers(0, 256, (ncw, N)).astype(np.uint8)
    hp = torch.from_numpy(h.copy()).pin_memory().numpy()
    # the host side shares its cores and memory bus with whatever else runs on the box: seven
    # repetitions each, the median reported and the spread beside it
    e2e, spread = {}, {}
    for name, buf in (("pageable", h), ("pinned", hp)):
        codec.encode_host(buf, K)
        codec.decode_host(buf, K)
        rates = []
        for _ in range(7):
            t1 = time.perf_counter()
            codec.encode_host(buf, K)
            r = codec.decode_host(buf, K)
            rates.append(ncw * N / (time.perf_counter() - t1) / 1e9)
            assert (r == 0).all()
        e2e[name] = round(float(np.median(rates)), 3)
        spread[name] = [round(min(rates), 3), round(max(rates), 3)]
    # decode of a pinned batch with 1 % of the rows corrupted (2 symbol errors each): those rows
    # come back over PCIe
    idx = np.arange(0, ncw, 100)
    ref = hp.copy()
    rates = []
    for _ in range(7):
        hp[idx, 7] ^= 0x5A
        hp[idx, 200] ^= 0xA5
        t1 = time.perf_counter()
        r = codec.decode_host(hp, K)
        rates.append(ncw * N / (time.perf_counter() - t1) / 1e9)
        assert int((r != 0).sum()) == len(idx) and np.array_equal(hp, ref)
    e2e["pinned_decode_1pct_corrupted"] = round(float(np.median(rates)), 3)
    spread["pinned_decode_1pct_corrupted"] = [round(min(rates), 3), round(max(rates), 3)]
    out["e2e_host_gbs"] = e2e
    out["e2e_host_spread_gbs"] = spread
    log(f"extras: e2e {e2e}")
    return out


def bench_shards(args):
    """SURVEY.md 8d C2 shard batches: S-byte shards (S = 1 KiB .. 1 MiB) in the rsencode layout
    (rsencode.C:93-163: 223-byte chunks, each followed by its 32 parity bytes, the last chunk
    shortened), ~256 MB of shard data per GPU (device-resident).  The whole batch is one
    ezrs_encode_shards and one ezrs_decode_shards call (one launch of the tile kernels each; the
    shortened rows are handled inside them).  Per S the line reports the encode+decode rate of
    shard bytes and each call's HBM fraction."""
    import torch
    import ezrs
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    torch.cuda.set_device(local)
    codec = ezrs.Codec.rs(N, K, device=local)
    gen = torch.Generator(device="cuda").manual_seed(0x5EED0003)
    sweep = []
    for S in (1 << 10, 1 << 14, 1 << 18, 1 << 20):
        sweep.append(shard_point(codec, S, args.steps, args.warmup, gen))
        log(f"shards S={S}: {sweep[-1]}")
    best = max(sweep, key=lambda r: r["gbs_shard_data"])
    print(json.dumps({"metric": "RS(255,223) shard-batch encode+decode GB/s device-resident (sweep)",
                      "value": best["gbs_shard_data"], "unit": "GB/s", "n_gpus": world,
                      "steps": args.steps, "warmup": args.warmup, "higher_is_better": True,
                      "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
                      "config": {"workload": "C2 shard batches: S-byte shards (rsencode layout), "
                                             "~256 MB per step, one call per direction",
                                 "codec": "RS(255,223) poly 0x11d fcr 1 prim 1"},
                      "sweep": sweep}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000,
                    help="timed steps (default 1000, ~0.18 s for C2: a timed region starts from an "
                         "idle GPU -- the synchronize before it -- and carries a fixed ~2 ms while "
                         "the clocks come back up; r04v: 100 steps 1371 GB/s, 400 1468, 1000 1496)")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--spinup", type=float, default=0.5,
                    help="seconds of untimed device spin-up (whole steps) before the counted warm-up")
    ap.add_argument("--ncw", type=int, default=1 << 20, help="codewords per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=3.0,
                    help="seconds per CPU-baseline measurement (5 configs x 1/all threads)")
    ap.add_argument("--e2e", action="store_true", help="also time the host-memory pipeline")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the extra figures of the default N=1 C2 run (shards 1 KiB / 1 MiB, "
                         "C2 at 4M codewords, C3 decode, host-memory rates)")
    ap.add_argument("--workload", choices=("c2", "c1", "c3", "c4", "c5", "shards"), default="c2",
                    help="c2: the headline RS(255,223) line; c1: the same for RS(255,251); c3: "
                         "RS(255,223) 8 errors + 4 erasures decode; c4: RS(65535,65503); c5: "
                         "BCH(1023,983,4) (SURVEY.md 8d); shards: RS(255,223) over S-byte shards, "
                         "S = 1 KiB .. 1 MiB (rsencode layout, one call per direction)")
    ap.add_argument("--k", type=int, default=0,
                    help="c2 workload with another RS(255,K) codec (the plane-sliced set: "
                         "NROOTS <= 32); the headline is K = 223")
    ap.add_argument("--share-gpus", action="store_true",
                    help="let ranks share GPUs when --gpus exceeds the visible devices (the "
                         "one-GPU harness test); the line is then marked, never a scaling run")
    ap.add_argument("--harness-check", action="store_true",
                    help="CPU/gloo check of the multi-rank harness (placeholder step, no GPU)")
    args = ap.parse_args()
    global SHARE_GPUS
    SHARE_GPUS = args.share_gpus
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_distributed(args))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        log(f"bench: note: WORLD_SIZE={os.environ['WORLD_SIZE']} ranks, --gpus {args.gpus}")
    if args.harness_check:
        return harness_check(args)
    if args.workload == "c5":
        return bench_c5(args)
    if args.workload in ("c3", "c4"):
        return bench_rs_errors(args)
    if args.workload == "shards":
        return bench_shards(args)

    import torch
    import torch.distributed as dist
    import ezrs
    import shard

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = bench_device(local)
    if world > 1:
        dist.init_process_group("gloo")

    n, k = (255, 251) if args.workload == "c1" else (N, args.k or K)
    enc_bytes, dec_bytes = n, n + 4               # encode: k read + n-k written; decode: n read + result
    codec = ezrs.Codec.rs(n, k, device=local)
    ncw = args.ncw
    codec.reserve(ncw)
    gen = torch.Generator(device="cuda").manual_seed(0x5EED0002 + rank)
    cw = torch.randint(0, 256, (ncw, n), generator=gen, device="cuda", dtype=torch.int32)
    cw = cw.to(torch.uint8)
    result = torch.empty(ncw, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()

    def step():
        codec.encode(cw, k, stream=stream)
        codec.decode(cw, k, result=result, stream=stream)

    # untimed device spin-up before the W counted warm-up steps: r05a probe (tools/step_probe.py)
    # -- in a fresh process the first ~50 steps run 10-25 % slower (0.23 -> 0.195 -> 0.18 ms) while
    # the GPU settles, which a 20-step timed region after 5 warm-up steps would carry; the spin-up is
    # reported on the line ("spinup_s")
    t_spin = time.perf_counter()
    while time.perf_counter() - t_spin < args.spinup:
        for _ in range(25):
            step()
        torch.cuda.synchronize()
    spinup_s = time.perf_counter() - t_spin
    for _ in range(args.warmup):
        step()

    # the timed region: K steps back to back, no event records between the calls (each record is
    # a few microseconds of GPU-timeline barrier -- r04l kernel trace: 5.8 us per record, ~7 % of a
    # step); the wall clock between two synchronizes gives value and ms_per_step.  The clean-decode
    # check runs after it: between the warm-up and the timed region the GPU only drains (a check
    # there idles it for ~2 ms, and the clocks then ramp back up inside the timed region -- r04w:
    # 100 steps 1370 GB/s whatever the warm-up, 1000 steps 1496)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = shard.max_over_ranks(elapsed)
    bad = int((result != 0).sum())
    if bad:
        raise SystemExit(f"rank {rank}: {bad} encoded codewords did not decode clean")
    # per-call averages for the roofline: 25 untimed steps are enqueued first (the check above
    # idled the GPU; they cover the ~2 ms clock ramp, so the first event is recorded on a busy GPU),
    # then KC = max(K, 200) encodes and KC (clean) decodes of the same batch back to back, bracketed
    # by three HIP events on the launch stream, one synchronize at the end (r05k: with K = 20 and 3
    # untimed steps the decode average read 0.086 ms against the kernel trace's 0.072)
    for _ in range(25):
        step()
    kc = max(args.steps, 200)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record(stream)
    for _ in range(kc):
        codec.encode(cw, k, stream=stream)
    ev[1].record(stream)
    for _ in range(kc):
        codec.decode(cw, k, result=result, stream=stream)
    ev[2].record(stream)
    ev[2].synchronize()
    enc_ms = ev[0].elapsed_time(ev[1]) / kc
    dec_ms = ev[1].elapsed_time(ev[2]) / kc

    total_cw = ncw * world * args.steps
    value = total_cw * n / elapsed / 1e9
    if enc_ms >= dec_ms:
        dom, ms, per_cw = "ezrs_encode", enc_ms, enc_bytes
    else:
        dom, ms, per_cw = "ezrs_decode", dec_ms, dec_bytes
    achieved = ncw * per_cw / (ms * 1e-3) / 1e9
    roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": load_traffic(args.workload, dom, ncw), "kernel": dom,
                "algorithmic_bytes_per_launch": ncw * per_cw,
                "avg_ms": {"ezrs_encode": round(enc_ms, 4), "ezrs_decode": round(dec_ms, 4)},
                "avg_calls": kc}

    e2e = None
    if args.e2e and rank == 0:
        import numpy as np
        h = np.random.default_rng(3).integers(0, 256, (ncw, n)).astype(np.uint8)
        # pinned (page-locked, hipHostMalloc via torch) copy of the same batch: the north_star's
        # "pinned hipMemcpyAsync" end-to-end rate; the pageable numpy rate is reported beside it
        hp = torch.from_numpy(h.copy()).pin_memory().numpy()
        e2e = {}
        for name, buf in (("pageable", h), ("pinned", hp)):
            codec.encode_host(buf, k)              # warm-up: staging buffers sized by both calls
            codec.decode_host(buf, k)
            rates = []
            for _ in range(7):                       # median of seven: the host is shared
                t1 = time.perf_counter()
                codec.encode_host(buf, k)
                r = codec.decode_host(buf, k)
                rates.append(ncw * n / (time.perf_counter() - t1) / 1e9)
                assert (r == 0).all()
            e2e[name] = round(float(np.median(rates)), 3)
            log(f"host-memory ({name}) encode+decode: {e2e[name]} GB/s")

    extras = None
    if world == 1 and args.workload == "c2" and not args.k and not args.no_extras:
        extras = c2_extras(codec, args)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baselines(args.cpu_seconds)

    if rank == 0:
        line = {"metric": f"RS({n},{k}) encode+decode GB/s device-resident",
                "value": round(value, 3), "unit": "GB/s", **gpu_fields(world), "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
                "higher_is_better": True, "vs_baseline": None, "spinup_s": round(spinup_s, 3),
                "dtype": "u8", "data": "synthetic",
                "config": {"workload": f"{args.workload.upper()}: RS({n},{k}) encode + clean decode, "
                                       f"{ncw} codewords/GPU",
                           "codec": f"RS({n},{k}) poly 0x11d fcr 1 prim 1",
                           "codewords_per_gpu": ncw, "global_codewords": ncw * world,
                           "bytes_per_codeword": n, "parallelism": f"shard{world}"},
                "roofline": roofline, "cpu_baseline": cpu}
        if e2e is not None:
            line["e2e_host_gbs"] = e2e
        if extras is not None:
            line.update(extras)
            # the dominant call's fraction past the 256 MiB Infinity Cache: the same calls on 4 M
            # codewords (1.07 GB) in this run, the HBM figure (the 1 M batch is 267 MB, which the
            # L3 partly serves)
            c4m = extras["c2_4m"]
            roofline["past_l3"] = {"codewords": c4m["codewords"],
                                   "frac_encode": c4m["frac_encode"], "frac_decode": c4m["frac_decode"],
                                   "frac": c4m["frac_encode"] if dom == "ezrs_encode" else c4m["frac_decode"]}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
