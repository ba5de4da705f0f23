"""The other Newton systems on the GPU (Settings, SymbolicOptimization.h:
28-64): one-sided / absent variable and inequality bounds and
InequalityHandling::Slacks (with the reference's corrector defect), through
the C ABI, against the reference's own Newton traces (tests/golden/
{vlo,vup,vnone,alo,aup,vlo0,sl,slbox}_*, and for the equality handlings and
NaiveSlacks {reg,pen,naive,naivereg,eqss}_*, made by tests/golden/
make_golden.py) and against the oracle at blocked-factor sizes.

Tolerances as tests/test_gpu_parity.py: element-wise formulas (initial
iterate, KKT assembly) bit-identical; directions 1e-9 relative per block and
||dx_gpu - dx_ref||_inf < 1e-10 (BASELINE.json north_star)."""
import numpy as np
import pytest

import oracle
from golden_io import load, sym_from_lower, trace

pytestmark = pytest.mark.gpu

I = pytest.importorskip("ipmz_amd")

DX_TOL = 1e-10
ABI_BOUNDS = {3: I.BOUNDS_BOTH, 1: I.BOUNDS_LOWER, 2: I.BOUNDS_UPPER, 0: I.BOUNDS_NONE}

# (tag, n, m, oracle.Form(slacks, inequality bounds mask, variable bounds mask)),
# as tests/test_oracle_golden.py FORMS
FORMS = [
    ("vlo", 48, 16, oracle.Form(False, 3, 1)), ("vup", 48, 16, oracle.Form(False, 3, 2)),
    ("vnone", 48, 16, oracle.Form(False, 3, 0)), ("alo", 48, 16, oracle.Form(False, 1, 3)),
    ("aup", 48, 16, oracle.Form(False, 2, 3)), ("vlo0", 48, 0, oracle.Form(False, 0, 1)),
    ("sl", 48, 16, oracle.Form(True, 3, 3)), ("slbox", 48, 0, oracle.Form(True, 0, 3)),
]


@pytest.fixture(scope="module")
def ctx():
    return I.Context(0)


def _abi(form):
    return dict(inequality_handling=I.INEQ_SLACKS if form.slacks else I.INEQ_SLACKED_SLACKS,
                inequality_bounds=ABI_BOUNDS[form.ineq_bounds], variable_bounds=ABI_BOUNDS[form.var_bounds])


def _close(got, ref, label):
    scale = max(1.0, np.abs(ref).max())
    assert np.abs(got - ref).max() < 1e-9 * scale, label


@pytest.mark.parametrize("tag,n,m,form", FORMS, ids=[f[0] for f in FORMS])
def test_formulation_golden_trace(ctx, tag, n, m, form):
    names, rows, conv = trace(tag)
    g = I.Optimizer(n, m, 0, ctx, **_abi(form))
    g.generate(7)
    assert g.state_len == len(load(f"{tag}_it0_vars.bin"))
    # initial iterate and KKT assembly: element-wise, bit for bit
    assert np.array_equal(g.vars(), load(f"{tag}_it0_vars.bin"))
    assert np.array_equal(g.kkt(), np.tril(sym_from_lower(load(f"{tag}_it0_kkt.bin"), n + m)))
    o = oracle.OracleQP(oracle.gen_qp(n, m, 0, 7), form=form)
    for it, ref in enumerate(rows):
        g.set_vars(load(f"{tag}_it{it}_vars.bin"))
        s0 = g.scalars()
        for k in ("f", "res", "mu"):
            assert abs(s0[k] - ref[k]) <= 1e-12 * max(1.0, abs(ref[k])), (tag, it, k, s0[k], ref[k])
        g.step()
        s1 = g.scalars()
        for k in ("alpha_aff", "mu_aff", "sigma", "alpha"):
            assert abs(s1[k] - ref[k]) <= 1e-9 * max(1.0, abs(ref[k])), (tag, it, k, s1[k], ref[k])
        for got, which in ((g.daff(), "daff"), (g.dir(), "d")):
            want = load(f"{tag}_it{it}_{which}.bin")
            so, sg = o.split(want), o.split(got)
            for s in o.order:
                _close(sg[s], so[s], (tag, it, which, s))
            assert np.abs(sg["x"] - so["x"]).max() < DX_TOL, (tag, it, which)
        if it + 1 < len(rows):  # the update: v + 0.995 alpha d, element-wise
            _close(g.vars(), load(f"{tag}_it{it + 1}_vars.bin"), (tag, it, "update"))


@pytest.mark.parametrize("tag,form", [(f[0], f[3]) for f in FORMS], ids=[f[0] for f in FORMS])
def test_formulation_blocked_vs_oracle(ctx, tag, form):
    # past one diagonal block (nbi = 64) and with equality rows (Regularization)
    n, m, p, seed = 300, (0 if tag in ("vlo0", "slbox") else 70), 30, 3
    o = oracle.OracleQP(oracle.gen_qp(n, m, p, seed), form=form)
    g = I.Optimizer(n, m, p, ctx, **_abi(form))
    g.generate(seed)
    assert np.array_equal(g.vars(), o.vars())
    assert np.array_equal(g.kkt(), np.tril(o.kkt()))
    for it in range(4):
        s0 = g.scalars()
        done, rec = o.iterate()
        for k in ("f", "res", "mu"):
            assert abs(s0[k] - rec[k]) <= 1e-12 * max(1.0, abs(rec[k])), (tag, it, k)
        if done:
            break
        g.step()
        s1 = g.scalars()
        for k in ("alpha_aff", "mu_aff", "sigma", "alpha"):
            assert abs(s1[k] - rec[k]) <= 1e-9 * max(1.0, abs(rec[k])), (tag, it, k, s1[k], rec[k])
        for which, (a, b) in enumerate(((g.daff(), o.daff()), (g.dir(), o.dir()))):
            sa, sb = o.split(a), o.split(b)
            for s in o.order:
                _close(sa[s], sb[s], (tag, it, which, s))
            assert np.abs(sa["x"] - sb["x"]).max() < DX_TOL, (tag, it, which)
        g.set_vars(o.vars())


def test_formulation_batch_matches_single(ctx):
    n, m, B = 96, 24, 3
    form = dict(inequality_handling=I.INEQ_SLACKED_SLACKS, inequality_bounds=I.BOUNDS_LOWER,
                variable_bounds=I.BOUNDS_UPPER)
    bt = I.Batch(n, m, 0, B, ctx, **form)
    bt.generate(11)
    bt.step()
    g = I.Optimizer(n, m, 0, ctx, **form)
    g.generate(12)  # QP 1 of the batch uses seed + 1
    g.step()
    sc = g.scalars()
    import torch
    dst = torch.zeros(B * I.SC_COUNT, dtype=torch.float64, device="cuda")
    bt.copy_batch_scalars(dst.data_ptr())
    torch.cuda.synchronize()
    ref = dst.cpu().numpy().reshape(B, I.SC_COUNT)
    for k in ("alpha_aff", "alpha", "mu_aff"):
        assert abs(ref[1, I.SC[k]] - sc[k]) <= 1e-12 * max(1.0, abs(sc[k])), k


@pytest.mark.parametrize("kw,msg", [
    (dict(inequality_bounds=3), "m > 0 with no inequality bound"),
    (dict(inequality_handling=1, variable_bounds=1), "Slacks with one-sided bounds"),
    (dict(inequality_handling=2, inequality_bounds=1), "NaiveSlacks with one-sided inequality bounds"),
    (dict(inequality_handling=3), "unknown inequality handling"),
    (dict(variable_bounds=4), "unknown bounds"),
])
def test_formulation_rejected(ctx, kw, msg):
    with pytest.raises(I.IpmzError):
        I.Optimizer(16, 4, 0, ctx, **kw)


# Equality rows and the other handlings against the reference's own Newton
# iterations (make_golden.py "reg" = C3's structure, "pen", "naive",
# "naivereg", "eqss"; the harness expands only the scalar blocks the
# reference's evaluate_matrix asserts on).  From the reference's iterate each
# iteration: scalars, both directions per block, the update.
EQ_CASES = [
    ("reg", 8, dict(), lambda qp: oracle.OracleQP(qp)),
    ("pen", 8, dict(equality_handling=I.EQ_PENALTY), lambda qp: oracle.OracleQP(qp, eq_penalty=True)),
    ("pex", 8, dict(equality_handling=I.EQ_PENALTY_EXTRA_DUAL), lambda qp: oracle.OracleQP(qp, eq_penalty=True)),
    ("naive", 0, dict(inequality_handling=I.INEQ_NAIVE_SLACKS),
     lambda qp: oracle.OracleQP(qp, form=oracle.Form(naive=True))),
    ("naivereg", 8, dict(inequality_handling=I.INEQ_NAIVE_SLACKS),
     lambda qp: oracle.OracleQP(qp, form=oracle.Form(naive=True))),
    ("eqss", 8, dict(equality_handling=I.EQ_SLACKED_SLACKS), oracle.EqSlackedOracle),
    ("naiveeq", 8, dict(inequality_handling=I.INEQ_NAIVE_SLACKS, equality_handling=I.EQ_NAIVE_SLACKS),
     lambda qp: oracle.EqSlackedOracle(qp, naive=True)),
]


def _kkt_ref_order(g, o):
    # the device KKT (lower triangle, the step's row order) in the reference's
    # row order (EqSlackedOracle.kperm: NaiveSlacks equality rows interleave)
    K = np.tril(g.kkt())
    K = K + np.tril(K, -1).T
    kp = getattr(o, "kperm", np.arange(K.shape[0]))
    return np.tril(K[np.ix_(kp, kp)])


@pytest.mark.parametrize("tag,p,kw,mk", EQ_CASES, ids=[c[0] for c in EQ_CASES])
def test_equality_golden_trace(ctx, tag, p, kw, mk):
    n, m = 48, 16
    fx = "pen" if tag == "pex" else tag  # PenaltyFunctionWithExtraDual: the same Newton system
    names, rows, conv = trace(fx)
    o = mk(oracle.gen_qp(n, m, p, 7))
    g = I.Optimizer(n, m, p, ctx, **kw)
    g.generate(7)
    assert g.state_len == len(load(f"{fx}_it0_vars.bin")) and g.N == o.N
    assert np.array_equal(g.vars(), load(f"{fx}_it0_vars.bin"))
    assert np.array_equal(_kkt_ref_order(g, o), np.tril(sym_from_lower(load(f"{fx}_it0_kkt.bin"), o.N)))
    for it, ref in enumerate(rows):
        g.set_vars(load(f"{fx}_it{it}_vars.bin"))
        s0 = g.scalars()
        for k in ("f", "res", "mu"):
            assert abs(s0[k] - ref[k]) <= 1e-12 * max(1.0, abs(ref[k])), (tag, it, k, s0[k], ref[k])
        g.step()
        s1 = g.scalars()
        for k in ("alpha_aff", "mu_aff", "sigma", "alpha"):
            assert abs(s1[k] - ref[k]) <= 1e-9 * max(1.0, abs(ref[k])), (tag, it, k, s1[k], ref[k])
        for got, which in ((g.daff(), "daff"), (g.dir(), "d")):
            so, sg = o.split(load(f"{fx}_it{it}_{which}.bin")), o.split(got)
            for s in o.order:
                _close(sg[s], so[s], (tag, it, which, s))
            assert np.abs(sg["x"] - so["x"]).max() < DX_TOL, (tag, it, which)
        if it + 1 < len(rows):
            _close(g.vars(), load(f"{fx}_it{it + 1}_vars.bin"), (tag, it, "update"))
    g.set_vars(load(f"{fx}_it{len(rows) - 1}_vars.bin"))
    g.step()
    assert g.scalars()["converged"] == 1.0


# InequalityHandling::NaiveSlacks at blocked-factor sizes against the oracle
# (pinned above to the reference's iterations at n = 48)
@pytest.mark.parametrize("n,m,p,seed", [(48, 16, 6, 7), (300, 70, 30, 3)])
def test_naive_slacks_vs_oracle(ctx, n, m, p, seed):
    form = oracle.Form(naive=True)
    o = oracle.OracleQP(oracle.gen_qp(n, m, p, seed), form=form)
    g = I.Optimizer(n, m, p, ctx, inequality_handling=I.INEQ_NAIVE_SLACKS)
    g.generate(seed)
    assert g.N == n + 2 * m + p == o.N
    assert np.array_equal(g.vars(), o.vars())
    assert np.array_equal(g.kkt(), np.tril(o.kkt()))
    for it in range(8):
        s0 = g.scalars()
        done, rec = o.iterate()
        for k in ("f", "res", "mu"):
            assert abs(s0[k] - rec[k]) <= 1e-12 * max(1.0, abs(rec[k])), (it, k)
        if done:
            assert s0["converged"] == 1.0
            break
        g.step()
        s1 = g.scalars()
        for k in ("alpha_aff", "mu_aff", "sigma", "alpha"):
            assert abs(s1[k] - rec[k]) <= 1e-9 * max(1.0, abs(rec[k])), (it, k, s1[k], rec[k])
        for which, (a, b) in enumerate(((g.daff(), o.daff()), (g.dir(), o.dir()))):
            sa, sb = o.split(a), o.split(b)
            for s in o.order:
                _close(sa[s], sb[s], (it, which, s))
            assert np.abs(sa["x"] - sb["x"]).max() < DX_TOL, (it, which)
        g.set_vars(o.vars())


def test_naive_slacks_batch_and_solve(ctx):
    n, m, p, B = 64, 16, 8, 3
    bt = I.Batch(n, m, p, B, ctx, inequality_handling=I.INEQ_NAIVE_SLACKS)
    bt.generate(5)
    g = I.Optimizer(n, m, p, ctx, inequality_handling=I.INEQ_NAIVE_SLACKS)
    g.generate(6)  # QP 1 of the batch
    iters, tr = g.solve(100)
    assert tr[-1]["converged"] == 1.0 and iters < 40
    o = oracle.OracleQP(oracle.gen_qp(n, m, p, 6), form=oracle.Form(naive=True))
    for it in range(100):
        done, _ = o.iterate()
        if done:
            break
    assert iters == it
    assert np.abs(o.split(g.vars())["x"] - o.split(o.vars())["x"]).max() < 1e-8
    bt.step()
    with pytest.raises(I.IpmzError):
        g.set_reduction(I.REDUCTION_NORMAL)


# EqualityHandling::SlackedSlacks at blocked-factor sizes, in a batch, through
# the normal equations, and its state permutation
def _eqss_iterations(g, o, iters, label):
    for it in range(iters):
        s0 = g.scalars()
        done, rec = o.iterate()
        for k in ("f", "res", "mu"):
            assert abs(s0[k] - rec[k]) <= 1e-12 * max(1.0, abs(rec[k])), (label, it, k)
        if done:
            assert s0["converged"] == 1.0
            return
        g.step()
        s1 = g.scalars()
        for k in ("alpha_aff", "mu_aff", "sigma", "alpha"):
            assert abs(s1[k] - rec[k]) <= 1e-9 * max(1.0, abs(rec[k])), (label, it, k, s1[k], rec[k])
        for which, (a, b) in enumerate(((g.daff(), o.daff()), (g.dir(), o.dir()))):
            sa, sb = o.split(a), o.split(b)
            for s in o.order:
                _close(sa[s], sb[s], (label, it, which, s))
            assert np.abs(sa["x"] - sb["x"]).max() < DX_TOL, (label, it, which)
        g.set_vars(o.vars())


@pytest.mark.parametrize("n,m,p,seed", [(300, 70, 30, 3), (200, 0, 40, 4)])
def test_eq_slacked_slacks_vs_oracle(ctx, n, m, p, seed):
    o = oracle.EqSlackedOracle(oracle.gen_qp(n, m, p, seed))
    g = I.Optimizer(n, m, p, ctx, equality_handling=I.EQ_SLACKED_SLACKS)
    g.generate(seed)
    assert g.N == n + m + p == o.N and g.state_len == o.L
    assert np.array_equal(g.vars(), o.vars())
    assert np.array_equal(g.kkt(), np.tril(o.kkt()))
    _eqss_iterations(g, o, 5, "augmented")


def test_eq_slacked_slacks_normal_equations(ctx):
    n, m, p, seed = 160, 40, 24, 9
    o = oracle.EqSlackedOracle(oracle.gen_qp(n, m, p, seed))
    g = I.Optimizer(n, m, p, ctx, equality_handling=I.EQ_SLACKED_SLACKS)
    g.generate(seed)
    g.set_reduction(I.REDUCTION_NORMAL)
    _eqss_iterations(g, o, 4, "normal")


def test_eq_slacked_slacks_state_order(ctx):
    n, m, p = 40, 6, 5
    g = I.Optimizer(n, m, p, ctx, equality_handling=I.EQ_SLACKED_SLACKS)
    g.generate(2)
    o = oracle.EqSlackedOracle(oracle.gen_qp(n, m, p, 2))
    sp = o.split(g.vars())
    assert np.all(sp["t"] == 1.0) and np.all(sp["lambda_v"] == 1.0) and np.all(sp["w"] == 1.0)
    v = np.arange(g.state_len, dtype=np.float64) + 0.5  # set -> get is the identity in the reference's order
    g.set_vars(v)
    assert np.array_equal(g.vars(), v)


def test_eq_slacked_slacks_batch_and_solve(ctx):
    n, m, p, B = 64, 16, 8, 3
    kw = dict(equality_handling=I.EQ_SLACKED_SLACKS)
    bt = I.Batch(n, m, p, B, ctx, **kw)
    bt.generate(5)
    g = I.Optimizer(n, m, p, ctx, **kw)
    g.generate(6)  # QP 1 of the batch
    assert np.array_equal(bt.state(1), g.vars())
    bt.step()
    g.step()
    ref = bt.batch_scalars()
    sc = g.scalars()
    for k in ("alpha_aff", "alpha", "mu_aff"):
        assert abs(ref[1, I.SC[k]] - sc[k]) <= 1e-12 * max(1.0, abs(sc[k])), k
    assert np.abs(bt.state(1) - g.vars()).max() < 1e-12
    g.generate(6)
    iters, tr = g.solve(100)
    assert tr[-1]["converged"] == 1.0
    o = oracle.EqSlackedOracle(oracle.gen_qp(n, m, p, 6))
    for it in range(100):
        done, _ = o.iterate()
        if done:
            break
    assert iters == it
    sg = o.split(g.vars())
    assert np.abs(sg["x"] - o.split(o.vars())["x"]).max() < 1e-8
    qp = oracle.gen_qp(n, m, p, 6)
    assert np.abs(qp["C"] @ sg["x"] - qp["d"]).max() < 1e-7  # C x = d at the optimum


@pytest.mark.parametrize("kw", [dict(inequality_handling=1), dict(inequality_handling=2),
                                dict(inequality_bounds=1)])
def test_eq_slacked_slacks_rejected(ctx, kw):
    with pytest.raises(I.IpmzError):
        I.Optimizer(16, 4, 2, ctx, equality_handling=I.EQ_SLACKED_SLACKS, **kw)


# EqualityHandling::NaiveSlacks (with NaiveSlacks inequalities) at blocked
# sizes, in a batch, and its state order (pinned above to the reference's
# "naiveeq" iterations at n = 48)
@pytest.mark.parametrize("n,m,p,seed", [(300, 70, 30, 3), (200, 0, 40, 4)])
def test_eq_naive_slacks_vs_oracle(ctx, n, m, p, seed):
    kw = dict(inequality_handling=I.INEQ_NAIVE_SLACKS, equality_handling=I.EQ_NAIVE_SLACKS)
    o = oracle.EqSlackedOracle(oracle.gen_qp(n, m, p, seed), naive=True)
    g = I.Optimizer(n, m, p, ctx, **kw)
    g.generate(seed)
    assert g.N == n + 2 * (m + p) == o.N and g.state_len == o.L
    assert np.array_equal(g.vars(), o.vars())
    assert np.array_equal(_kkt_ref_order(g, o), np.tril(o.kkt()))
    _eqss_iterations(g, o, 5, "naive")


def test_eq_naive_slacks_state_order_batch_and_solve(ctx):
    n, m, p = 64, 16, 8
    kw = dict(inequality_handling=I.INEQ_NAIVE_SLACKS, equality_handling=I.EQ_NAIVE_SLACKS)
    g = I.Optimizer(n, m, p, ctx, **kw)
    g.generate(6)
    o = oracle.EqSlackedOracle(oracle.gen_qp(n, m, p, 6), naive=True)
    sp = o.split(g.vars())
    assert np.all(sp["v"] == 1.0) and np.all(sp["lambda_w"] == 1.0)
    v0 = g.vars()
    v = np.arange(g.state_len, dtype=np.float64) + 0.5  # set -> get is the identity in the reference's order
    g.set_vars(v)
    assert np.array_equal(g.vars(), v)
    g.set_vars(v0)
    iters, tr = g.solve(100)
    for it in range(100):
        done, _ = o.iterate()
        if done:
            break
    assert tr[-1]["converged"] == 1.0 and iters == it
    assert np.abs(o.split(g.vars())["x"] - o.split(o.vars())["x"]).max() < 1e-8
    bt = I.Batch(n, m, p, 3, ctx, **kw)
    bt.generate(5)  # QP 1 of the batch = seed 6
    for _ in range(3):
        bt.step()
    g2 = I.Optimizer(n, m, p, ctx, **kw)
    g2.generate(6)
    for _ in range(3):
        g2.step()
    assert np.abs(bt.state(1, 0) - g2.vars()).max() < 1e-12
    with pytest.raises(I.IpmzError):  # equality NaiveSlacks rides on NaiveSlacks inequalities
        I.Optimizer(n, m, p, ctx, equality_handling=I.EQ_NAIVE_SLACKS)
