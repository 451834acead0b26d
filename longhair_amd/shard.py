"""Stripe sharding across ranks (one process per GPU).

Stripes are independent, so the multi-GPU codec is a partition of the
stripe range with no collective on the data path.  These helpers are what bench.py and
the multi-process tests use; they work with the gloo (CPU) and nccl (RCCL) backends.
"""
import os


def world_info():
    """(world_size, rank, local_rank) from the torchrun environment (1, 0, 0 if absent)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(total, world, rank):
    """Contiguous [lo, hi) stripe range of `rank`; sizes differ by at most one stripe."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _reduce(value, op, device):
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(value, device="cpu"):
    """Slowest rank's value (elapsed times are reduced with MAX)."""
    import torch.distributed as dist
    return _reduce(value, dist.ReduceOp.MAX, device)


def sum_over_ranks(value, device="cpu"):
    import torch.distributed as dist
    return _reduce(value, dist.ReduceOp.SUM, device)


def aggregate_rate(bytes_this_rank, elapsed_this_rank, device="cpu"):
    """Whole-job throughput: every rank's bytes divided by the slowest rank's time."""
    total = sum_over_ranks(bytes_this_rank, device)
    slowest = max_over_ranks(elapsed_this_rank, device)
    return total / slowest
