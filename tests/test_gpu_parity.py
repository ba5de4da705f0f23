"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle
and the reference's golden vectors.  Run on an MI355X: pytest -m gpu.

Tolerances
  * element-wise Newton formulas: bit-identical (same operand order,
    -ffp-contract=off) -- checked on KKT assembly and the initial iterate;
  * LDL^T inside one diagonal block (N <= nbi): bit-identical to the
    reference (same k-order of subtractions);
  * blocked factor / solve / matvec reductions: the target of BASELINE.json,
    ||dx_gpu - dx_cpu||_inf < 1e-10, plus relative checks on every block.
"""
import numpy as np
import pytest

import oracle
from golden_io import load, sym_from_lower, trace, unpack_lower

pytestmark = pytest.mark.gpu

I = pytest.importorskip("ipmz_amd")

DX_TOL = 1e-10  # BASELINE.json north_star: ||dx_gpu - dx_cpu||_inf < 1e-10


@pytest.fixture(scope="module")
def ctx():
    return I.Context(0)


# ---------------------------------------------------------------------------
# LinearSolvers (LinearSolvers.cpp:14-74)
@pytest.mark.parametrize("N,tag", [(8, "ldlt8"), (64, "ldlt64"), (320, "ldlt320")])
def test_ldlt_decomposition_golden(ctx, N, tag):
    K = sym_from_lower(load(f"{tag}_K.bin"), N)
    L_ref = unpack_lower(load(f"{tag}_L.bin"), N)
    D_ref = load(f"{tag}_D.bin")
    L, D, info = I.LinearSolvers.ldlt_decomposition(K, ctx)
    assert info == 0
    if N <= 64:  # one diagonal block: the reference's k-order of updates (fused multiply-adds)
        np.testing.assert_allclose(D, D_ref, rtol=1e-15, atol=0)
        assert np.abs(L - L_ref).max() < 1e-15 * max(1.0, np.abs(L_ref).max())
    else:
        np.testing.assert_allclose(D, D_ref, rtol=1e-13, atol=0)
        assert np.abs(L - L_ref).max() < 1e-13 * max(1.0, np.abs(L_ref).max())
    b = load(f"{tag}_b.bin")
    x_ref = load(f"{tag}_x.bin")
    x = I.LinearSolvers.overwriting_solve_ldlt(L_ref, D_ref, b.copy(), ctx)
    assert np.abs(x - x_ref).max() < 1e-12 * max(1.0, np.abs(x_ref).max())


def test_ldlt_zero_pivot_rule(ctx):
    K = np.array([[0.0, 1.0], [1.0, 2.0]])
    L, D, info = I.LinearSolvers.ldlt_decomposition(K, ctx)
    assert D[0] == 1e-8 and L[1, 0] == 1e8 and info == 0


def test_solve_empty_noop(ctx):
    b = np.zeros(0)
    I.LinearSolvers.overwriting_solve_ldlt(np.zeros((0, 0)), np.zeros(0), b, ctx)


def test_non_square_raises(ctx):
    with pytest.raises(I.IpmzError):
        I.LinearSolvers.ldlt_decomposition(np.zeros((3, 4)), ctx)


def _qd(N, seed):
    rng = np.random.default_rng(seed)
    n1 = (3 * N + 3) // 4
    K = rng.uniform(-1, 1, (N, N))
    K[:n1, :n1] /= n1
    K[n1:, :n1] /= np.sqrt(n1)
    K[n1:, n1:] = 0
    K = np.tril(K) + np.tril(K, -1).T  # symmetric
    d = rng.uniform(0.5, 1.5, N)
    K[np.arange(n1), np.arange(n1)] = 1 + d[:n1]
    K[np.arange(n1, N), np.arange(n1, N)] = -d[n1:]
    return K


@pytest.mark.parametrize("N", [127, 129, 300, 513, 1000])
@pytest.mark.parametrize("blocking", [(256, 64), (256, 128), (128, 64), (512, 128), (512, 64)])
def test_ldlt_ragged_vs_oracle(ctx, N, blocking):
    ctx.set_blocking(*blocking)
    try:
        K = _qd(N, N)
        L_o, D_o = oracle.ldlt(K)
        L, D, info = I.LinearSolvers.ldlt_decomposition(K, ctx)
        assert info == 0
        assert np.abs(D - D_o).max() < 1e-12 * np.abs(D_o).max()
        assert np.abs(L - L_o).max() < 1e-11 * max(1.0, np.abs(L_o).max())
        b = np.random.default_rng(1).uniform(-1, 1, N)
        x_o = oracle.solve_ldlt(L_o, D_o, b)
        x = I.LinearSolvers.overwriting_solve_ldlt(L, D, b.copy(), ctx)
        assert np.abs(x - x_o).max() < 1e-10
    finally:
        ctx.set_blocking(256, 64)


# ---------------------------------------------------------------------------
# Newton step (Optimizer.cpp:127-219) vs the oracle, re-synchronised to the
# oracle's iterate after every step so each comparison starts from the same
# point.
def _compare_dirs(o, g, label):
    split_o = o.split(o.daff()), o.split(o.dir())
    split_g = o.split(g.daff()), o.split(g.dir())
    for which in (0, 1):
        for s in o.order:
            a, b = split_g[which][s], split_o[which][s]
            scale = max(1.0, np.abs(b).max())
            err = np.abs(a - b).max()
            assert err < 1e-9 * scale, (label, which, s, err)
        assert np.abs(split_g[which]["x"] - split_o[which]["x"]).max() < DX_TOL, (label, which)


@pytest.mark.parametrize("n,m,p,seed", [(64, 0, 0, 1234), (48, 16, 0, 7), (256, 64, 0, 0), (64, 16, 8, 1234),
                                        (300, 70, 30, 3), (700, 150, 60, 9)])
def test_newton_steps_vs_oracle(ctx, n, m, p, seed):
    qp = oracle.gen_qp(n, m, p, seed)
    o = oracle.OracleQP(qp)
    g = I.Optimizer(n, m, p, ctx)
    g.generate(seed)
    # generator + build_environment + assembly are element-wise: bitwise
    assert np.array_equal(g.vars(), o.vars())
    assert np.array_equal(g.kkt(), np.tril(o.kkt()))
    for it in range(6):
        s0 = g.scalars()
        done, rec = o.iterate()
        for k in ("f", "res", "mu"):
            assert abs(s0[k] - rec[k]) <= 1e-12 * max(1.0, abs(rec[k])), (it, k, s0[k], rec[k])
        if done:
            assert s0["converged"] == 1.0
            break
        g.step()
        s1 = g.scalars()
        for k in ("alpha_aff", "mu_aff", "sigma", "alpha"):
            assert abs(s1[k] - rec[k]) <= 1e-9 * max(1.0, abs(rec[k])), (it, k, s1[k], rec[k])
        _compare_dirs(o, g, f"iter {it}")
        g.set_vars(o.vars())


def test_newton_golden_c4_directions(ctx):
    # C4-size QP (n=256, m=64) directly against the reference's own vectors
    names, rows, _ = trace("c4")
    g = I.Optimizer(256, 64, 0, ctx)
    g.generate(0)
    for it in range(len(rows)):
        v_ref = load(f"c4_it{it}_vars.bin")
        g.set_vars(v_ref)
        g.step()
        for got, tag in ((g.daff(), "daff"), (g.dir(), "d")):
            ref = load(f"c4_it{it}_{tag}.bin")
            assert np.abs(got - ref).max() < 1e-9 * max(1.0, np.abs(ref).max()), (it, tag)
            assert np.abs(got[:256] - ref[:256]).max() < DX_TOL, (it, tag)
        s = g.scalars()
        assert abs(s["alpha"] - rows[it]["alpha"]) < 1e-9


@pytest.mark.parametrize("tag,n,m,seed", [("c1", 64, 0, 1234), ("s1", 48, 16, 7)])
def test_full_solve_matches_reference_trace(ctx, tag, n, m, seed):
    names, rows, conv = trace(tag)
    g = I.Optimizer(n, m, 0, ctx)
    g.generate(seed)
    iters, tr = g.solve(100)
    assert iters == conv
    for it, ref in enumerate(rows):
        for k in ("f", "res", "mu"):
            assert abs(tr[it][k] - ref[k]) <= 1e-8 * max(1.0, abs(ref[k])), (it, k)


def test_load_host_matches_generate(ctx):
    n, m, p, seed = 96, 24, 12, 5
    qp = oracle.gen_qp(n, m, p, seed)
    d = I.Data(qp["Q"], qp["c"], qp["lx"], qp["ux"], qp["A"], qp["lA"], qp["uA"], qp["C"], qp["d"])
    a = I.Optimizer.from_data(d, ctx)
    b = I.Optimizer(n, m, p, ctx)
    b.generate(seed)
    assert np.array_equal(a.kkt(), b.kkt())
    assert np.array_equal(a.residuals(), b.residuals())


def test_build_environment_validation(ctx):
    # EnvironmentBuilder.cpp:12-17: l_x < u_x and l_A <= u_A are asserted
    n = 4
    d = I.Data(np.eye(n), np.zeros(n), np.ones(n), np.ones(n))
    with pytest.raises(I.IpmzError, match="l_x < u_x"):
        I.Optimizer.from_data(d, ctx)


def test_regularization_solve_converges(ctx):
    g = I.Optimizer(200, 50, 20, ctx)
    g.generate(11)
    iters, tr = g.solve(100)
    assert tr[-1]["converged"] == 1.0 and iters < 40
    o = oracle.OracleQP(oracle.gen_qp(200, 50, 20, 11))
    for _ in range(100):
        done, _ = o.iterate()
        if done:
            break
    assert np.abs(g.vars() - o.vars()).max() < 1e-6


# ---------------------------------------------------------------------------
# Full-size properties (BASELINE.json configs) -- the oracle cannot factor
# these in test time; size-independent checks instead.
def test_c3_size_converges_and_solves(ctx):
    n, m, p = 8192, 2048, 1024  # C3: N = 11264
    g = I.Optimizer(n, m, p, ctx)
    g.generate(1234)
    iters, tr = g.solve(60)
    assert tr[-1]["converged"] == 1.0, tr[-1]
    assert tr[-1]["res"] < 1e-8 and tr[-1]["mu"] < 1e-8
    # monotone decrease of mu over the solve (predictor-corrector behaviour)
    mus = [r["mu"] for r in tr]
    assert mus[-1] < 1e-8 < mus[0]


def test_large_factor_residual(ctx):
    torch = pytest.importorskip("torch")
    N = 6000
    K = torch.from_numpy(_qd(N, 77)).cuda()
    Kf = K.clone()
    ld = N
    D = torch.zeros(N, dtype=torch.float64, device="cuda")
    wsb = ctx.workspace_bytes(N)
    ws = torch.zeros(wsb // 8 + 1, dtype=torch.float64, device="cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        info = ctx.ldlt_factor(N, Kf.data_ptr(), ld, D.data_ptr(), ws.data_ptr(), wsb)
        assert info == 0
        b = torch.rand(N, dtype=torch.float64, device="cuda") * 2 - 1
        x = b.clone()
        ctx.ldlt_solve(N, Kf.data_ptr(), ld, D.data_ptr(), ws.data_ptr(), x.data_ptr())
        torch.cuda.synchronize()
        r = K @ x - b
        rel = (r.abs().max() / (K.abs().max() * x.abs().max())).item()
        assert rel < 1e-13, rel
    finally:
        ctx.set_stream(None)
