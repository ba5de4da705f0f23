"""Normal-equations reduction (BASELINE config C2) through the C ABI.

The reference only builds the normal equations symbolically
(SymbolicOptimization.cpp:465-478); its numeric path solves the augmented
system.  The oracle for this reduction is therefore the reference's
augmented Newton direction (same mathematics) -- the
golden C4-size vectors and the CPU oracle -- and, for the bare factor/solve,
an fp64 numpy solve of the same augmented matrix.  Expected deviation is
cond(S)-scaled rounding; the BASELINE bound ||dx_gpu - dx_cpu||_inf < 1e-10
is asserted on the Newton directions.
"""
import numpy as np
import pytest

import oracle
from golden_io import load, trace

pytestmark = pytest.mark.gpu
I = pytest.importorskip("ipmz_amd")
torch = pytest.importorskip("torch")
DX_TOL = 1e-10


@pytest.fixture(scope="module")
def ctx():
    c = I.Context(0)
    c.set_stream(torch.cuda.current_stream().cuda_stream)
    yield c
    c.set_stream(None)


def _aug(n, mp, seed, spd_h=True):
    rng = np.random.default_rng(seed)
    H = rng.uniform(-1, 1, (n, n)) / n
    H = np.tril(H) + np.tril(H, -1).T
    H[np.arange(n), np.arange(n)] = rng.uniform(1, 2, n) * (1 if spd_h else np.where(np.arange(n) == n // 2, -1, 1))
    B = rng.uniform(-1, 1, (mp, n)) / np.sqrt(n)
    E = rng.uniform(0.5, 1.5, mp)
    K = np.zeros((n + mp, n + mp))
    K[:n, :n] = H
    K[n:, :n] = B
    K[:n, n:] = B.T
    K[n:, n:] = -np.diag(E)
    return K


def _normal(ctx, K, n, b):
    N = K.shape[0]
    mp = N - n
    Kd = torch.from_numpy(np.tril(K)).cuda()
    D = torch.zeros(N, dtype=torch.float64, device="cuda")
    wsb = ctx.normal_workspace_bytes(n, mp)
    ws = torch.zeros(wsb // 8 + 1, dtype=torch.float64, device="cuda")
    info = ctx.normal_factor(n, mp, Kd.data_ptr(), N, D.data_ptr(), ws.data_ptr(), wsb)
    if info:
        return info, None, None
    x = torch.from_numpy(b.copy()).cuda()
    ctx.normal_solve(n, mp, Kd.data_ptr(), N, D.data_ptr(), ws.data_ptr(), x.data_ptr())
    torch.cuda.synchronize()
    return 0, x.cpu().numpy(), D.cpu().numpy()


@pytest.mark.parametrize("n,mp", [(64, 16), (100, 0), (300, 70), (1000, 250), (1024, 512)])
def test_normal_factor_solve_vs_numpy(ctx, n, mp):
    K = _aug(n, mp, n + mp)
    b = np.random.default_rng(5).uniform(-1, 1, n + mp)
    info, x, D = _normal(ctx, K, n, b)
    assert info == 0
    # pivots of H (> 0), then of -S, S = E + B H^-1 B^T SPD (the x-first
    # elimination: the augmented LDL^T's (2,2) pivots)
    assert (D[:n] > 0).all() and (D[n:] < 0).all()
    ref = np.linalg.solve(K, b)
    assert np.abs(x - ref).max() < 1e-12 * max(1.0, np.abs(ref).max())
    L, Dr, _ = I.LinearSolvers.ldlt_decomposition(K, ctx)
    assert np.allclose(D, Dr, rtol=1e-12)
    # S's pivots against an independent Cholesky of the explicitly formed S
    if 0 < mp <= 250:
        H, B, E = K[:n, :n], K[n:, :n], -np.diag(K[n:, n:])
        S = np.diag(E) + B @ np.linalg.solve(H, B.T)
        Ls = np.linalg.cholesky(S)
        assert np.allclose(-D[n:], np.diag(Ls) ** 2, rtol=1e-10)


def test_normal_rejects_indefinite_h(ctx):
    n, mp = 128, 32
    K = _aug(n, mp, 3, spd_h=False)
    info, _, _ = _normal(ctx, K, n, np.ones(n + mp))
    assert info >= 1 and info <= n  # first non-positive pivot lies in H


def _compare(o, g, n, label):
    for which, (a, b) in enumerate(((g.daff(), o.daff()), (g.dir(), o.dir()))):
        assert np.abs(a[:n] - b[:n]).max() < DX_TOL, (label, which)
        assert np.abs(a - b).max() < 1e-9 * max(1.0, np.abs(b).max()), (label, which)


@pytest.mark.parametrize("n,m,p,seed", [(64, 16, 8, 1234), (300, 70, 30, 3), (256, 64, 0, 0)])
def test_normal_newton_vs_oracle(ctx, n, m, p, seed):
    o = oracle.OracleQP(oracle.gen_qp(n, m, p, seed))
    g = I.Optimizer(n, m, p, ctx)
    g.generate(seed)
    g.set_reduction(I.REDUCTION_NORMAL)
    for it in range(5):
        done, rec = o.iterate()
        if done:
            break
        g.step()
        _compare(o, g, n, f"iter {it}")
        s = g.scalars()
        assert abs(s["alpha"] - rec["alpha"]) <= 1e-9 * max(1.0, abs(rec["alpha"]))
        g.set_vars(o.vars())


def test_normal_golden_c4(ctx):
    # the reference's own augmented directions at iterates 0..3 (n=256, m=64)
    names, rows, _ = trace("c4")
    g = I.Optimizer(256, 64, 0, ctx)
    g.generate(0)
    g.set_reduction(I.REDUCTION_NORMAL)
    for it in range(len(rows)):
        g.set_vars(load(f"c4_it{it}_vars.bin"))
        g.step()
        for tag, got in (("daff", g.daff()), ("d", g.dir())):
            ref = load(f"c4_it{it}_{tag}.bin")
            assert np.abs(got[:256] - ref[:256]).max() < DX_TOL, (it, tag)


def test_c2_size_normal_matches_augmented(ctx):
    # C2: n = 2048, m = 512 -- same iteration count and solution as the
    # augmented reduction (size-independent properties)
    n, m = 2048, 512
    ga = I.Optimizer(n, m, 0, ctx)
    ga.generate(1234)
    ia, ta = ga.solve(60)
    gn = I.Optimizer(n, m, 0, ctx)
    gn.generate(1234)
    gn.set_reduction(I.REDUCTION_NORMAL)
    inn, tn = gn.solve(60)
    assert tn[-1]["converged"] == 1.0 and ia == inn
    assert np.abs(gn.vars()[:n] - ga.vars()[:n]).max() < 1e-7
