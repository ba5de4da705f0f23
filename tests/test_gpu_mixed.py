"""Mixed precision (BASELINE config C5): fp32 LDL^T of the scaled KKT matrix
+ fp64 iterative refinement, through the C ABI, against fp64 references.

Tolerance sweep: for tol in 1e-6 .. 1e-12 the refinement must stop with
||b - K x||_inf <= tol ||b||_inf (checked again here in fp64 with numpy), and
the solution error must follow the residual: ||x - x_ref||_inf <=
cond-scaled tol.  Newton directions through the mixed solve are compared
with the CPU oracle (the reference algorithm, fp64): at the tightest
tolerance the BASELINE bound ||dx_gpu - dx_cpu||_inf < 1e-10 holds.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu
I = pytest.importorskip("ipmz_amd")
torch = pytest.importorskip("torch")

TOLS = [1e-6, 1e-8, 1e-10, 1e-12]


@pytest.fixture(scope="module")
def ctx():
    c = I.Context(0)
    c.set_stream(torch.cuda.current_stream().cuda_stream)
    yield c
    c.set_stream(None)


def _qd(N, seed, spd=False):
    """Quasi-definite (or SPD) symmetric test matrix, lower triangle used."""
    rng = np.random.default_rng(seed)
    n1 = N if spd else (3 * N + 3) // 4
    K = rng.uniform(-1, 1, (N, N))
    K[:n1, :n1] /= n1
    K[n1:, :n1] /= np.sqrt(n1)
    K[n1:, n1:] = 0
    K = np.tril(K) + np.tril(K, -1).T
    d = rng.uniform(0.5, 1.5, N)
    K[np.arange(n1), np.arange(n1)] = 1 + d[:n1]
    K[np.arange(n1, N), np.arange(n1, N)] = -d[n1:]
    # badly scaled rows/columns: what S = diag(|K_ii|^-1/2) is for
    sc = np.exp(rng.uniform(-1.5, 1.5, N))
    return K * sc[:, None] * sc[None, :]


def _mixed(ctx, K, b, tol, max_refine=30):
    N = K.shape[0]
    Kd = torch.from_numpy(np.tril(K)).cuda()
    wsb = ctx.mixed_workspace_bytes(N)
    ws = torch.zeros(wsb // 8 + 1, dtype=torch.float64, device="cuda")
    info = ctx.mixed_factor(N, Kd.data_ptr(), N, ws.data_ptr(), wsb)
    assert info == 0
    x = torch.from_numpy(b.copy()).cuda()
    ratio, iters = ctx.mixed_solve(N, Kd.data_ptr(), N, ws.data_ptr(), x.data_ptr(), tol, max_refine)
    torch.cuda.synchronize()
    # K itself is left intact (the residual needs it)
    assert np.array_equal(Kd.cpu().numpy(), np.tril(K))
    return x.cpu().numpy(), ratio, iters


@pytest.mark.parametrize("N,spd", [(100, True), (300, False), (1000, False), (2500, True)])
def test_mixed_solve_tolerance_sweep(ctx, N, spd):
    K = _qd(N, 11 + N, spd)
    b = np.random.default_rng(N).uniform(-1, 1, N)
    x_ref = np.linalg.solve(K, b)
    cond = np.linalg.cond(K)
    prev = None
    for tol in TOLS:
        x, ratio, iters = _mixed(ctx, K, b, tol)
        r = np.abs(b - K @ x).max() / np.abs(b).max()
        assert ratio <= tol and r <= 2 * tol, (tol, ratio, r, iters)
        err = np.abs(x - x_ref).max() / np.abs(x_ref).max()
        assert err <= 10 * cond * tol + 1e-13, (tol, err, cond)
        if prev is not None:
            assert iters >= prev  # tighter tolerance, at least as many corrections
        prev = iters
    # fp32 factor alone (no correction) is ~1e-7-accurate relative to fp64
    x0, ratio0, it0 = _mixed(ctx, K, b, 1e-30, max_refine=0)
    assert it0 == 0 and ratio0 > 1e-12


def _box_qp_dirs(ctx, n, m, p, seed, tol, max_refine=30):
    qp = oracle.gen_qp(n, m, p, seed)
    o = oracle.OracleQP(qp)
    g = I.Optimizer(n, m, p, ctx)
    g.generate(seed)
    g.set_mixed_precision(True, tol, max_refine)
    return o, g


@pytest.mark.parametrize("n,m,p,seed", [(512, 0, 0, 1234), (300, 70, 30, 3)])
def test_mixed_newton_directions_vs_oracle(ctx, n, m, p, seed):
    o, g = _box_qp_dirs(ctx, n, m, p, seed, 1e-14)
    for it in range(4):
        done, rec = o.iterate()
        if done:
            break
        g.step()
        torch.cuda.synchronize()
        dx = np.abs(g.dir()[:n] - o.dir()[:n]).max()
        dxa = np.abs(g.daff()[:n] - o.daff()[:n]).max()
        assert dx < 1e-10 and dxa < 1e-10, (it, dx, dxa)
        s = g.scalars()
        assert abs(s["alpha"] - rec["alpha"]) <= 1e-9 * max(1.0, abs(rec["alpha"]))
        g.set_vars(o.vars())


def test_mixed_newton_tolerance_sweep(ctx):
    # ||dx_gpu - dx_cpu||_inf tracks the refinement tolerance
    n, seed = 512, 1234
    errs = []
    for tol in TOLS:
        o, g = _box_qp_dirs(ctx, n, 0, 0, seed, tol)
        o.iterate()
        g.step()
        s = g.scalars()
        assert s["ir_ratio"] <= tol and s["ir_ratio_aff"] <= tol
        errs.append(np.abs(g.dir()[:n] - o.dir()[:n]).max())
    assert errs[-1] < 1e-10, errs
    assert errs[0] > errs[-1], errs


def test_c5_size_converges_mixed(ctx):
    # C5: n = 16384 box-only, fp32 factor + fp64 refinement; size-independent
    # properties: the IPM converges and every solve met its tolerance
    n = 16384
    g = I.Optimizer(n, 0, 0, ctx)
    g.generate(1234)
    g.set_mixed_precision(True, 1e-12, 20)
    iters, tr = g.solve(60)
    assert tr[-1]["converged"] == 1.0, tr[-1]
    s = g.scalars()
    assert s["ir_ratio"] <= 1e-12 and s["ir_ratio_aff"] <= 1e-12
