"""EqualityHandling::None on the GPU (§8f row f3): the zero (lambda_C,
lambda_C) block the reference routes to solve_indefinite_
(Optimizer.cpp:63-75, ASSERT(false) there), solved with the Bunch-Kaufman
factor (bk.hip, bitwise to LinearSolvers.cpp:76-207) inside the same
on-device Newton step.  Oracle: the CPU restatement (oracle eq_none=True;
component-pinned, see tests/test_oracle_eqnone.py)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
I = pytest.importorskip("ipmz_amd")
DX_TOL = 1e-10


@pytest.fixture(scope="module")
def ctx():
    return I.Context(0)


def _compare(o, g, label):
    for got, ref in ((g.daff(), o.daff()), (g.dir(), o.dir())):
        so, sg = o.split(ref), o.split(got)
        for s in o.order:
            err = np.abs(sg[s] - so[s]).max()
            assert err < 1e-9 * max(1.0, np.abs(so[s]).max()), (label, s, err)
        assert np.abs(sg["x"] - so["x"]).max() < DX_TOL, label


@pytest.mark.parametrize("n,m,p,seed", [(40, 10, 6, 3), (64, 16, 8, 1234), (30, 0, 4, 9), (300, 60, 40, 2)])
def test_newton_steps_vs_oracle(ctx, n, m, p, seed):
    o = oracle.OracleQP(oracle.gen_qp(n, m, p, seed), eq_none=True)
    g = I.Optimizer(n, m, p, ctx, equality_handling=I.EQ_NONE)
    g.generate(seed)
    assert np.array_equal(g.vars(), o.vars())
    assert np.array_equal(g.kkt(), np.tril(o.kkt()))  # zero block included, bitwise
    for it in range(5):
        s0 = g.scalars()
        done, rec = o.iterate()
        for k in ("f", "res", "mu"):
            assert abs(s0[k] - rec[k]) <= 1e-12 * max(1.0, abs(rec[k])), (it, k)
        if done:
            break
        g.step()
        s1 = g.scalars()
        for k in ("alpha_aff", "mu_aff", "sigma", "alpha"):
            assert abs(s1[k] - rec[k]) <= 1e-9 * max(1.0, abs(rec[k])), (it, k)
        _compare(o, g, f"iter {it}")
        g.set_vars(o.vars())


def test_full_solve_same_iterations(ctx):
    n, m, p, seed = 64, 16, 8, 1234
    o = oracle.OracleQP(oracle.gen_qp(n, m, p, seed), eq_none=True)
    for it in range(100):
        done, _ = o.iterate()
        if done:
            break
    g = I.Optimizer(n, m, p, ctx, equality_handling=I.EQ_NONE)
    g.generate(seed)
    iters, tr = g.solve(100)
    assert iters == it and tr[-1]["converged"] == 1.0
    assert np.abs(g.vars() - o.vars()).max() < 1e-8


def test_batch_vs_oracle(ctx):
    n, m, p, B, seed0 = 48, 12, 6, 5, 40
    bt = I.Batch(n, m, p, B, ctx, equality_handling=I.EQ_NONE)
    bt.generate(seed0)
    orcs = [oracle.OracleQP(oracle.gen_qp(n, m, p, seed0 + i), eq_none=True) for i in range(B)]
    for it in range(3):
        for o in orcs:
            o.iterate()
        bt.step()
        for i, o in enumerate(orcs):
            got, ref = bt.state(i, 2), o.dir()
            assert np.abs(got - ref).max() < 1e-9 * max(1.0, np.abs(ref).max()), (it, i)
            assert np.abs(got[:n] - ref[:n]).max() < DX_TOL, (it, i)
            bt.set_state(i, o.vars())


@pytest.mark.parametrize("n,m,p,seed,iters", [(900, 120, 60, 5, 2), (4096, 512, 256, 7, 1)])
def test_newton_steps_grid_factor_vs_oracle(ctx, n, m, p, seed, iters):
    # N = 1080 and 4864: the whole-device Bunch-Kaufman factor (bk.hip
    # k_bk_grid, IPMZ_BK_GRID_MIN = 512), the second beyond one workgroup's
    # former N <= 4096 limit
    o = oracle.OracleQP(oracle.gen_qp(n, m, p, seed), eq_none=True)
    g = I.Optimizer(n, m, p, ctx, equality_handling=I.EQ_NONE)
    g.generate(seed)
    for it in range(iters):
        done, rec = o.iterate()
        assert not done
        g.step()
        s1 = g.scalars()
        for k in ("alpha_aff", "mu_aff", "sigma", "alpha"):
            assert abs(s1[k] - rec[k]) <= 1e-9 * max(1.0, abs(rec[k])), (it, k)
        _compare(o, g, f"iter {it}")
        g.set_vars(o.vars())


def test_limits_and_exclusions(ctx):
    with pytest.raises(I.IpmzError, match="Bunch-Kaufman"):  # batches: one workgroup per system
        I.Batch(4000, 100, 10, 2, ctx, equality_handling=I.EQ_NONE)
    g = I.Optimizer(32, 8, 4, ctx, equality_handling=I.EQ_NONE)
    with pytest.raises(I.IpmzError):
        g.set_reduction(I.REDUCTION_NORMAL)
    with pytest.raises(I.IpmzError):
        g.set_mixed_precision(True)


# ---------------------------------------------------------------------------
# EqualityHandling::PenaltyFunction (§8f row f4): -mu (lambda_C, lambda_C)
# block (mu = the environment's mu at assembly), r_lambda_C carries mu; the
# reference's evaluator asserts on the scalar block (Evaluation.cpp:57-60).
@pytest.mark.parametrize("n,m,p,seed", [(40, 10, 6, 3), (300, 60, 40, 2)])
def test_penalty_newton_steps_vs_oracle(ctx, n, m, p, seed):
    o = oracle.OracleQP(oracle.gen_qp(n, m, p, seed), eq_penalty=True)
    g = I.Optimizer(n, m, p, ctx, equality_handling=I.EQ_PENALTY)
    g.generate(seed)
    assert np.array_equal(g.vars(), o.vars())
    assert np.array_equal(g.kkt(), np.tril(o.kkt()))  # -mu block with mu = 1 at the start
    for it in range(5):
        done, rec = o.iterate()
        if done:
            break
        g.step()
        s1 = g.scalars()
        for k in ("alpha_aff", "mu_aff", "sigma", "alpha"):
            assert abs(s1[k] - rec[k]) <= 1e-9 * max(1.0, abs(rec[k])), (it, k)
        _compare(o, g, f"iter {it}")
        g.set_vars(o.vars())


def test_penalty_full_solve(ctx):
    n, m, p, seed = 64, 16, 8, 1234
    o = oracle.OracleQP(oracle.gen_qp(n, m, p, seed), eq_penalty=True)
    for it in range(100):
        done, _ = o.iterate()
        if done:
            break
    g = I.Optimizer(n, m, p, ctx, equality_handling=I.EQ_PENALTY)
    g.generate(seed)
    iters, tr = g.solve(100)
    assert iters == it and tr[-1]["converged"] == 1.0
    assert np.abs(g.vars() - o.vars()).max() < 1e-8


def test_penalty_extra_dual_matches_penalty(ctx):
    # IPMZ_EQ_PENALTY_EXTRA_DUAL: the reference's PenaltyFunctionWithExtraDual
    # system is PenaltyFunction's (tests/test_oracle_eqnone.py): bit for bit
    n, m, p, seed = 48, 12, 6, 4
    a = I.Optimizer(n, m, p, ctx, equality_handling=I.EQ_PENALTY)
    b = I.Optimizer(n, m, p, ctx, equality_handling=I.EQ_PENALTY_EXTRA_DUAL)
    a.generate(seed)
    b.generate(seed)
    for _ in range(3):
        a.step()
        b.step()
        assert np.array_equal(a.vars(), b.vars()) and np.array_equal(a.dir(), b.dir())

