"""A stuck cross-workgroup hand-off must surface as an error, never as a
silently wrong success (sync.h: every spin is bounded at 0.5 s and raises a
sticky error word; capi.cpp folds those words into the return codes).

The hand-off is broken on purpose with the ipmz_debug_inject test hook: the
persistent kernels then drop their first publication, so every consumer
times out."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
I = pytest.importorskip("ipmz_amd")
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    return I.Context(0)


def _qd(N, seed=5):
    rng = np.random.default_rng(seed)
    K = rng.uniform(-1, 1, (N, N)) / N
    K = np.tril(K) + np.tril(K, -1).T
    K[np.arange(N), np.arange(N)] = 1.0 + rng.uniform(size=N)
    return K


def test_newton_step_solve_timeout_raises(ctx):
    g = I.Optimizer(300, 60, 20, ctx)
    g.generate(3)
    I.debug_inject(I.INJECT_SOLVE)
    try:
        g.step()
        with pytest.raises(I.IpmzError, match="timed out"):
            g.scalars()
    finally:
        I.debug_inject(0)
    # the next factorization clears the sticky word: a clean step succeeds
    g.generate(3)
    g.step()
    assert np.isfinite(g.scalars()["alpha"])


def test_factor_panel_timeout_raises(ctx):
    N = 700  # three outer panels: the fused outer-panel kernel runs
    K = torch.from_numpy(_qd(N)).cuda()
    D = torch.zeros(N, dtype=torch.float64, device="cuda")
    wsb = ctx.workspace_bytes(N)
    ws = torch.zeros(wsb // 8 + 1, dtype=torch.float64, device="cuda")
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        I.debug_inject(I.INJECT_PANEL)
        try:
            with pytest.raises(I.IpmzError, match="outer-panel"):
                ctx.ldlt_factor(N, K.clone().data_ptr(), N, D.data_ptr(), ws.data_ptr(), wsb)
        finally:
            I.debug_inject(0)
        Kf = K.clone()
        assert ctx.ldlt_factor(N, Kf.data_ptr(), N, D.data_ptr(), ws.data_ptr(), wsb) == 0
        # a solve timeout is reported by the next ipmz_ctx_sync
        x = torch.ones(N, dtype=torch.float64, device="cuda")
        I.debug_inject(I.INJECT_SOLVE)
        try:
            ctx.ldlt_solve(N, Kf.data_ptr(), N, D.data_ptr(), ws.data_ptr(), x.data_ptr())
        finally:
            I.debug_inject(0)
        with pytest.raises(I.IpmzError, match="triangular solve"):
            ctx.sync()
    finally:
        ctx.set_stream(None)


def test_host_signature_solve_timeout_raises(ctx):
    """ipmz_overwriting_solve_ldlt (the reference's host signature) frees its
    workspace before returning: a solve timeout must be reported by that call
    itself, and a later ipmz_ctx_sync must not read the freed workspace."""
    N = 300
    K = _qd(N, 9)
    L, D, info = I.LinearSolvers.ldlt_decomposition(K, ctx)
    assert info == 0
    b = np.ones(N)
    I.debug_inject(I.INJECT_SOLVE)
    try:
        with pytest.raises(I.IpmzError, match="triangular solve"):
            I.LinearSolvers.overwriting_solve_ldlt(L, D, b.copy(), ctx)
    finally:
        I.debug_inject(0)
    ctx.sync()  # nothing pending: the timeout was already reported
    x = I.LinearSolvers.overwriting_solve_ldlt(L, D, b.copy(), ctx)
    assert np.abs(K @ x - b).max() < 1e-10
