"""The panel's chain roles factor bitwise alike whichever launch runs them
(panel.hip): the chain launch (production), every chain role run by the
rows launch (debug bit IPMZ_DEBUG_ROWS_CHAIN: no chain launch at all -- what
a serialized dispatch order, e.g. under rocprofv3 --pmc, produces), and the
early chain launch's give-back (debug bit IPMZ_DEBUG_GIVEBACK: a chain
launch started beside the previous panel's rows launch never sees that
launch's RDONE flags, so prev_rows_ready times out after 1 ms, the launch
draws no role and the rows launch queued behind it takes every chain role;
N <= 4096 left from a panel), and the same give-back on the panel's
READY-TO-FACTOR word (debug bit IPMZ_DEBUG_READY_LATE: the B stream raises it
3 ms late, so the chain launch sees RDONE[0] but not the word -- the branch a
serialized dispatch took when it timed out in round 6).  A role may land in either launch, so the
forms must agree to the bit or the factor would not be run-to-run
deterministic, and no form may raise the sticky hand-off error.

fp64 (LinearSolvers::ldlt_decomposition, LinearSolvers.cpp:14-42, blocked,
look-ahead schedule) and the fp32 factor of the mixed-precision path."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
I = pytest.importorskip("ipmz_amd")
torch = pytest.importorskip("torch")

GIVEBACK, ROWS_CHAIN = 2048, 4096  # kernels.h IPMZ_DEBUG_GIVEBACK / IPMZ_DEBUG_ROWS_CHAIN
READY_LATE = 32768  # kernels.h IPMZ_DEBUG_READY_LATE
MODES = [0, GIVEBACK, ROWS_CHAIN, READY_LATE]


@pytest.fixture(scope="module")
def ctx():
    c = I.Context(0)
    c.set_stream(torch.cuda.current_stream().cuda_stream)
    yield c
    c.set_stream(None)


def _qd(N, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    n1 = (3 * N) // 4
    K = torch.rand(N, N, device="cuda", dtype=torch.float64, generator=g) * 2 - 1
    K[:n1, :n1] /= n1
    K[n1:, :n1] /= n1 ** 0.5
    K[n1:, n1:] = 0
    idx = torch.arange(N, device="cuda")
    d = torch.rand(N, device="cuda", dtype=torch.float64, generator=g) + 0.5
    K[idx[:n1], idx[:n1]] = 1 + d[:n1]
    K[idx[n1:], idx[n1:]] = -d[n1:]
    return torch.tril(K).contiguous()


def _with_mask(mask, fn):
    I.debug_inject(mask)
    try:
        return fn()
    finally:
        I.debug_inject(0)


@pytest.mark.parametrize("N", [200, 1408, 2560, 4100])
def test_fp64_chain_forms_bitwise(ctx, N):
    """N = 200: one outer panel with a ragged last block; 1408: 256-wide
    panels; 2560 (C2's order): 384-wide panels, ragged last panel; 4100:
    512-wide panels, ragged last panel."""
    K = _qd(N, 7 * N)
    wsb = ctx.workspace_bytes(N)
    ws = torch.zeros(wsb // 8 + 1, dtype=torch.float64, device="cuda")
    D = torch.zeros(N, dtype=torch.float64, device="cuda")
    b = torch.rand(N, dtype=torch.float64, device="cuda")

    def run():
        Kf = K.clone()
        assert ctx.ldlt_factor(N, Kf.data_ptr(), N, D.data_ptr(), ws.data_ptr(), wsb) == 0
        x = b.clone()
        ctx.ldlt_solve(N, Kf.data_ptr(), N, D.data_ptr(), ws.data_ptr(), x.data_ptr())
        ctx.sync()  # raises on a sticky hand-off error (IPMZ_ERR_HIP)
        return torch.tril(Kf, -1).cpu().numpy(), D.cpu().numpy(), x.cpu().numpy()

    out = [_with_mask(m, run) for m in MODES + [0]]
    assert np.isfinite(out[0][0]).all() and np.isfinite(out[0][2]).all()
    for r in range(1, len(out)):
        for w in range(3):
            assert np.array_equal(out[r][w], out[0][w]), (MODES + [0])[r]


@pytest.mark.parametrize("N", [1408, 4100])
def test_fp32_chain_forms_bitwise(ctx, N):
    K = _qd(N, 7 * N + 1)
    wsb = ctx.mixed_workspace_bytes(N)
    ws = torch.zeros(wsb // 4 + 64, dtype=torch.float32, device="cuda")
    ld32 = (N + 63) // 64 * 64
    doff = ((N * ld32 * 4 + 255) // 256 * 256) // 4  # D32 follows K32 (mixed_ws_carve)

    def run():
        ws.zero_()
        assert ctx.mixed_factor(N, K.data_ptr(), N, ws.data_ptr(), wsb) == 0
        torch.cuda.synchronize()
        L = torch.tril(ws[:N * ld32].view(N, ld32)[:, :N], -1)
        return L.cpu().numpy(), ws[doff:doff + N].cpu().numpy()

    out = [_with_mask(m, run) for m in MODES]
    assert np.isfinite(out[0][0]).all()
    for r in range(1, len(out)):
        assert np.array_equal(out[r][0], out[0][0]) and np.array_equal(out[r][1], out[0][1]), MODES[r]


def test_c2_normal_steps_giveback_bitwise(ctx):
    """C2 (n = 2048, m = 512, normal equations, N = 2560, 384-wide panels --
    every panel's chain launch starts early): Newton steps with every early
    chain launch giving its roles back equal the production steps bitwise."""
    def run():
        g = I.Optimizer(2048, 512, 0, ctx)
        g.generate(1234)
        g.set_reduction(I.REDUCTION_NORMAL)
        out = []
        for _ in range(3):
            g.step()
            out.append((g.vars(), g.dir()))
        g.close()
        return out

    a, b = run(), _with_mask(GIVEBACK, run)
    for (va, da), (vb, db) in zip(a, b):
        assert np.array_equal(va, vb) and np.array_equal(da, db)
