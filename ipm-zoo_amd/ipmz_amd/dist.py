"""Multi-GPU plumbing for batches of independent QPs.

One process per GPU; each rank owns a contiguous shard of the QPs (no
data-path collective).  The only exchange is the per-iteration convergence
summary {max res, max mu, unconverged count} -- the stopping rule
res < 1e-8 and mu < 1e-8 of Optimizer.cpp:124-135 (res, mu from
:240-268) in MAX-reducible form -- computed on the device by ONE kernel
(ipmz_batch_summary) and combined by ONE all-reduce (MAX): RCCL over xGMI
on the GPUs, gloo in the CPU tests.  Every rank stops at the same iteration:
when the reduced unconverged count is 0, i.e. when the converged count of
the whole job reaches the global batch size.
"""
import torch
import torch.distributed as dist

SUMMARY_LEN = 3  # [max res, max mu, unconverged count], all MAX-reduced


def pack_summary(res, mu, unconverged, device):
    """Local summary -> tensor (host-side steppers; the device Batch writes
    the same layout with Batch.summary_into)."""
    return torch.tensor([float(res), float(mu), float(unconverged)], dtype=torch.float64, device=device)


def reduce_summary(summary, group=None):
    """ONE all-reduce (MAX) of a packed summary, in place."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(summary, op=dist.ReduceOp.MAX, group=group)
    return summary


def shard(batch, world, rank):
    """Contiguous shard of QP indices [0, batch) owned by this rank."""
    per = (batch + world - 1) // world
    lo = min(batch, rank * per)
    return range(lo, min(batch, lo + per))


def solve_sharded(stepper, max_iter=100, group=None, device="cuda", flags=0):
    """Optimizer::solve over a batch sharded across the ranks of `group`
    (the f2 row of SURVEY.md §8f): step this rank's QPs until the
    all-reduced summary says every QP of the whole job converged, or
    max_iter.  A converged QP keeps its iterate (the device step freezes it),
    so ranks that finished early just wait in the collective.

    stepper: an ipmz_amd.Batch (or anything with summary_into(tensor) and
    step(flags)).  Returns (iterations, [max res, max mu, unconverged]) --
    identical on every rank."""
    buf = torch.zeros(SUMMARY_LEN, dtype=torch.float64, device=device)
    it = 0
    while True:
        stepper.summary_into(buf)
        reduce_summary(buf, group)
        s = buf.tolist()  # the one host round trip per iteration (the reference prints here too)
        if s[2] == 0.0 or it >= max_iter:
            return it, s
        stepper.step(flags)
        it += 1
