"""Multi-GPU decomposition of the batch path.

Every codeword is independent, so a batch of ``ncw`` codewords is split into contiguous per-rank
ranges, one process per GPU (torchrun; RCCL is the process group on the GPU box, gloo in the CPU
tests).  Each rank builds its own codec on its own device and touches only its range: there is no
data-path collective.  The only cross-rank traffic is the timing reduction (max over ranks) and,
optionally, the sum of per-rank outcome counts.
"""
from __future__ import annotations


def shard_range(ncw: int, world: int, rank: int) -> tuple[int, int]:
    """[lo, hi) of rank's codewords: contiguous, covering, sizes differing by at most one."""
    if world < 1 or not 0 <= rank < world or ncw < 0:
        raise ValueError(f"bad shard request ncw={ncw} world={world} rank={rank}")
    base, rem = divmod(ncw, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def _group_ready():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def max_over_ranks(x: float, device=None) -> float:
    """The largest x over all ranks (the timing rule of bench.py); x itself without a group.
    bench.py's group is gloo (CPU): the scalars never touch a device, so ranks can even share one
    GPU (tests/test_bench_gpu.py runs --gpus 2 on a one-GPU box)."""
    if not _group_ready():
        return float(x)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(counts, device=None) -> list[int]:
    """Element-wise sum of per-rank integer counts (e.g. clean / corrected / failed codewords)."""
    counts = [int(c) for c in counts]
    if not _group_ready():
        return counts
    import torch
    import torch.distributed as dist
    t = torch.tensor(counts, dtype=torch.int64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(v) for v in t.tolist()]
