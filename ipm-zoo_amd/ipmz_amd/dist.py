"""Multi-GPU plumbing for batches of independent QPs.

One process per GPU; each rank owns its own QPs (no data-path collective).
The only exchange is the per-iteration convergence summary: max residual
norm, max mu and the number of converged QPs, packed in one small tensor and
all-reduced (RCCL over xGMI on the GPUs, gloo in the CPU tests).
"""
import torch
import torch.distributed as dist

SUMMARY_LEN = 3  # [max res, max mu, converged count]


def pack_summary(res, mu, converged, device):
    """Local summary -> tensor; res/mu/converged may be tensors or floats."""
    out = torch.empty(SUMMARY_LEN, dtype=torch.float64, device=device)
    out[0] = res
    out[1] = mu
    out[2] = converged
    return out


def reduce_summary(summary, group=None):
    """All-reduce a packed summary in place: max of res and mu, sum of the
    converged count (two collectives on the same small buffer)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return summary
    dist.all_reduce(summary[:2], op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(summary[2:], op=dist.ReduceOp.SUM, group=group)
    return summary


def shard(batch, world, rank):
    """Contiguous shard of QP indices [0, batch) owned by this rank."""
    per = (batch + world - 1) // world
    lo = min(batch, rank * per)
    return range(lo, min(batch, lo + per))
