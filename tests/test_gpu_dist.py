"""The sharded convergence loop (ipmz_amd.dist.solve_sharded, SURVEY.md §8f
row f2) with the HIP batch solver: two ranks share the box's one GPU (gloo
carries the one all-reduce per iteration; the driver's 8-GPU run uses RCCL).
Each rank's shard must stop at the iteration the whole job converges, and
every QP must end exactly where a single-process batch solve leaves it."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

BATCH, N, M = 16, 64, 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "ipm-zoo_amd"))
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ipmz_amd as I
    from ipmz_amd.dist import shard, solve_sharded

    mine = shard(BATCH, world, rank)
    b = I.Batch(N, M, 0, len(mine), I.Context(0))
    b.generate(mine.start)
    dev = torch.zeros(3, dtype=torch.float64, device="cuda")

    class Host:  # summary on the device, reduced through gloo on the host
        def summary_into(self, t):
            b.summary_into(dev)
            b.ctx.sync()
            t.copy_(dev.cpu())

        def step(self, flags=0):
            b.step(flags)

    it, s = solve_sharded(Host(), 80, device="cpu")
    out[rank] = (it, s, [b.state(i).tolist() for i in range(len(mine))])
    dist.destroy_process_group()


def test_sharded_batch_solve_two_ranks_one_gpu():
    import ipmz_amd as I

    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    (it0, s0, v0), (it1, s1, v1) = out[0], out[1]
    assert it0 == it1 and s0 == s1 and s0[2] == 0.0
    ref = I.Batch(N, M, 0, BATCH, I.Context(0))
    ref.generate(0)
    it, nconv = ref.solve_all(80)
    assert nconv == BATCH and it == it0
    got = np.array(v0 + v1)
    exp = np.array([ref.state(i) for i in range(BATCH)])
    assert np.array_equal(got, exp)


def test_solve_sharded_batch_on_own_stream():
    """A Batch passed straight to solve_sharded while its context runs on its
    own (non-blocking) stream: the summary must be ordered before torch's
    stream reads it (a stale zero buffer would stop the loop at iteration 0)."""
    import ipmz_amd as I
    from ipmz_amd.dist import solve_sharded

    ctx = I.Context(0)  # the context's own stream, not torch's
    b = I.Batch(N, M, 0, BATCH, ctx)
    b.generate(0)
    it, s = solve_sharded(b, 80, device="cuda")
    ref = I.Batch(N, M, 0, BATCH, I.Context(0))
    ref.generate(0)
    it_ref, nconv = ref.solve_all(80)
    assert nconv == BATCH and s[2] == 0.0 and it == it_ref > 0
    for i in range(BATCH):
        assert np.array_equal(b.state(i), ref.state(i)), i
