"""Batched Newton steps (config C4: independent QPs, one launch per phase
for the whole batch) vs the CPU oracle and the reference golden vectors."""
import numpy as np
import pytest

import oracle
from golden_io import load, trace

pytestmark = pytest.mark.gpu
I = pytest.importorskip("ipmz_amd")
DX_TOL = 1e-10


@pytest.fixture(scope="module")
def ctx():
    return I.Context(0)


@pytest.mark.parametrize("kernel", ["auto", "one", "left"])
@pytest.mark.parametrize("n,m,p,B,seed0", [(64, 16, 0, 5, 100), (256, 64, 0, 12, 0), (96, 24, 8, 4, 7),
                                           (300, 60, 0, 3, 50), (700, 90, 10, 2, 60)])
def test_batch_steps_vs_oracle(ctx, n, m, p, B, seed0, kernel):
    """Every small-factor kernel (ragged last blocks: N = 80, 112, 360, 800)."""
    bt = I.Batch(n, m, p, B, ctx)
    if kernel != "auto":
        bt.set_factor_kernel({"one": I.Batch.FACTOR_ONE, "left": I.Batch.FACTOR_LEFT}[kernel])
    bt.generate(seed0)
    orcs = [oracle.OracleQP(oracle.gen_qp(n, m, p, seed0 + i)) for i in range(B)]
    for i, o in enumerate(orcs):
        assert np.array_equal(bt.state(i, 0), o.vars()), i
    for it in range(3):
        recs = [o.iterate()[1] for o in orcs]
        bt.step()
        sc = bt.batch_scalars()
        for i, o in enumerate(orcs):
            for which, ref in ((1, o.daff()), (2, o.dir())):
                got = bt.state(i, which)
                assert np.abs(got - ref).max() < 1e-9 * max(1.0, np.abs(ref).max()), (it, i, which)
                assert np.abs(got[:n] - ref[:n]).max() < DX_TOL, (it, i, which)
            assert abs(sc[i, I.SC["alpha"]] - recs[i]["alpha"]) < 1e-9
            bt.set_state(i, o.vars())


def test_batch_c4_golden(ctx):
    # QP 0 of a seed-0 batch is the reference's C4-size golden QP (n=256, m=64)
    names, rows, _ = trace("c4")
    bt = I.Batch(256, 64, 0, 8, ctx)
    bt.generate(0)
    for it in range(len(rows)):
        bt.set_state(0, load(f"c4_it{it}_vars.bin"))
        bt.step()
        for which, tag in ((1, "daff"), (2, "d")):
            ref = load(f"c4_it{it}_{tag}.bin")
            got = bt.state(0, which)
            assert np.abs(got[:256] - ref[:256]).max() < DX_TOL, (it, tag)


def test_batch_solve_all_matches_single(ctx):
    n, m, B = 128, 32, 6
    bt = I.Batch(n, m, 0, B, ctx)
    bt.generate(300)
    its, nconv = bt.solve_all(100)
    assert nconv == B
    for i in range(B):
        g = I.Optimizer(n, m, 0, ctx)
        g.generate(300 + i)
        g.solve(100)
        assert np.abs(bt.state(i, 0) - g.vars()).max() < 1e-7, i


def _data(q):
    return I.Data(q["Q"], q["c"], q["lx"], q["ux"], q["A"], q["lA"], q["uA"], q["C"], q["d"])


def test_batch_reload_host_needs_initialize(ctx):
    """ipmz_batch_load_host leaves the batch uninitialized: the kept KKT matrix
    K0 (off-diagonal part written once per data load) still holds the old data,
    so a step before ipmz_batch_initialize is refused (IPMZ_ERR_STATE) instead
    of factoring the old matrix; after it, every QP -- the reloaded one with
    data the batch never saw -- steps like its own oracle run."""
    n, m, B = 96, 24, 3
    bt = I.Batch(n, m, 0, B, ctx)
    qps = [oracle.gen_qp(n, m, 0, 700 + i) for i in range(B)]
    for i, q in enumerate(qps):
        bt.load_one(i, _data(q))
    bt.initialize()
    bt.step()
    qps[1] = oracle.gen_qp(n, m, 0, 9999)  # new data for QP 1
    bt.load_one(1, _data(qps[1]))
    with pytest.raises(I.IpmzError):
        bt.step()
    bt.initialize()
    orcs = [oracle.OracleQP(q) for q in qps]
    for it in range(2):
        for o in orcs:
            o.iterate()
        bt.step()
        for i, o in enumerate(orcs):
            for which, ref in ((1, o.daff()), (2, o.dir())):
                got = bt.state(i, which)
                assert np.abs(got[:n] - ref[:n]).max() < DX_TOL, (it, i, which)
            bt.set_state(i, o.vars())
    bt.close()
