"""world_size-2 gloo test of the multi-GPU path's only exchange: the
convergence summary of independent QPs (ipmz_amd/dist.py), with the CPU
oracle standing in for each rank's device solver."""
import os
import socket

import pytest
import torch.multiprocessing as mp

torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path[:0] = [os.path.join(repo, "oracle"), os.path.join(repo, "ipm-zoo_amd")]
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    from ipmz_amd.dist import pack_summary, reduce_summary, shard

    batch = 5
    mine = list(shard(batch, world, rank))
    qps = [oracle.OracleQP(oracle.gen_qp(24, 6, 0, seed)) for seed in mine]
    done = [False] * len(qps)
    history = []
    for it in range(40):
        res = mu = 0.0
        conv = 0
        for k, q in enumerate(qps):
            if not done[k]:
                d, rec = q.iterate()
                done[k] = bool(d)
                res, mu = max(res, rec["res"]), max(mu, rec["mu"])
            conv += int(done[k])
        s = reduce_summary(pack_summary(res, mu, conv, "cpu"))
        history.append(s.tolist())
        if s[2].item() == batch:
            break
    out[rank] = history
    dist.destroy_process_group()


def test_shard_covers_batch():
    from ipmz_amd.dist import shard
    for batch in (1, 5, 1024):
        for world in (1, 2, 3, 8):
            idx = [i for r in range(world) for i in shard(batch, world, r)]
            assert idx == list(range(batch))


def test_convergence_summary_allreduce_world2():
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "oracle")]
    import oracle

    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    h0, h1 = out[0], out[1]
    assert h0 == h1  # every rank sees the same reduced summary
    assert h0[-1][2] == 5  # all five QPs converged, counted across ranks
    # single-process reference of the same reduction
    qps = [oracle.OracleQP(oracle.gen_qp(24, 6, 0, s)) for s in range(5)]
    done = [False] * 5
    for it, row in enumerate(h0):
        res = mu = 0.0
        for k, q in enumerate(qps):
            if not done[k]:
                d, rec = q.iterate()
                done[k] = bool(d)
                res, mu = max(res, rec["res"]), max(mu, rec["mu"])
        assert row[0] == res and row[1] == mu and row[2] == sum(done)
