"""Multi-GPU orchestration for batch verification.

Records are independent, so the batch shards into contiguous per-rank ranges
with no data-path collective. torch.distributed (gloo, CPU tensors only) is
used for control: the barrier around the timed region, the max-over-ranks
time, and the AND of per-rank parity. One process per GPU; the HIP work itself
never goes through torch.
"""
from __future__ import annotations

import os


def env_rank():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def shard_range(n_total: int, rank: int, world: int, align: int = 64):
    """Contiguous [lo, hi) of rank in a batch of n_total records; boundaries are
    multiples of `align` so per-rank bitmap words concatenate without shifts."""
    per = -(-n_total // world)
    per = -(-per // align) * align
    lo = min(n_total, rank * per)
    hi = min(n_total, lo + per)
    return lo, hi


def init(world: int):
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            dist.init_process_group("gloo")


def barrier(world: int):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def all_true(ok: bool, world: int) -> bool:
    if world == 1:
        return ok
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t[0])


def sum_over_ranks(x: int, world: int) -> int:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t[0])


def finalize(world: int):
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
