"""world_size-2 gloo tests of the multi-GPU path:
the sharded convergence loop ipmz_amd.dist.solve_sharded -- one all-reduce
(MAX) of {max res, max mu, unconverged count} per iteration -- driven on the
CPU by an oracle-backed stepper (the device Batch implements the same two
methods; tests/test_gpu_dist.py runs it with the HIP solver)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

torch = pytest.importorskip("torch")

BATCH, N, M = 5, 24, 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class OracleShard:
    """Stepper protocol of solve_sharded over CPU-oracle QPs: converged QPs
    are frozen, as the device step freezes them."""

    def __init__(self, seeds):
        import oracle
        self.qps = [oracle.OracleQP(oracle.gen_qp(N, M, 0, s)) for s in seeds]
        self.recs = [None] * len(self.qps)
        self.done = [False] * len(self.qps)
        self.steps = 0
        for k, q in enumerate(self.qps):
            self._eval(k)

    def _eval(self, k):
        q = self.qps[k]
        res, mu = q.residual_norm(), q.mu()
        self.recs[k] = (res, mu)
        self.done[k] = res < 1e-8 and mu < 1e-8

    def summary_into(self, t):
        t[0] = max(r[0] for r in self.recs) if self.recs else 0.0
        t[1] = max(r[1] for r in self.recs) if self.recs else 0.0
        t[2] = float(sum(not d for d in self.done))

    def step(self, flags=0):
        self.steps += 1
        for k, q in enumerate(self.qps):
            if not self.done[k]:
                q.iterate()
                self._eval(k)


def _setup_paths():
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (here, os.path.join(repo, "oracle"), os.path.join(repo, "ipm-zoo_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _worker(rank, world, port, out):
    _setup_paths()
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ipmz_amd.dist import shard, solve_sharded
    from test_dist_gloo import OracleShard

    st = OracleShard(list(shard(BATCH, world, rank)))
    it, s = solve_sharded(st, 60, device="cpu")
    out[rank] = (it, s, [q.vars().tolist() for q in st.qps], st.steps)
    dist.destroy_process_group()


def test_shard_covers_batch():
    from ipmz_amd.dist import shard
    for batch in (1, 5, 1024):
        for world in (1, 2, 3, 8):
            idx = [i for r in range(world) for i in shard(batch, world, r)]
            assert idx == list(range(batch))


def test_sharded_solve_world2_matches_single_process():
    _setup_paths()
    from ipmz_amd.dist import solve_sharded

    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    (it0, s0, v0, n0), (it1, s1, v1, n1) = out[0], out[1]
    # every rank leaves the loop at the same iteration with the same reduced summary
    assert it0 == it1 == n0 == n1 and s0 == s1
    assert s0[2] == 0.0 and s0[0] < 1e-8 and s0[1] < 1e-8
    # the single-process loop over the whole batch gives the same answer
    ref = OracleShard(range(BATCH))
    it, s = solve_sharded(ref, 60, device="cpu")
    assert it == it0 and s == s0
    assert v0 + v1 == [q.vars().tolist() for q in ref.qps]  # bitwise: each QP's own iterates
