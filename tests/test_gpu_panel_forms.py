"""The panel's chain roles in both of their forms factor bitwise alike
(panel.hip): the 4-wave chain of the 256-thread chain launch (production),
the 8-wave chain of the 512-thread chain launch (debug bit IPMZ_DEBUG_CHAIN8), and
every chain role run by the rows launch in its 4-wave form (debug bit
IPMZ_DEBUG_ROWS_CHAIN -- what a serialized dispatch order, e.g. under
rocprofv3 --pmc, produces).  A role may land in either launch, so the forms
must agree to the bit or the factor would not be run-to-run deterministic.

fp64 (LinearSolvers::ldlt_decomposition, LinearSolvers.cpp:14-42, blocked,
look-ahead schedule) and the fp32 factor of the mixed-precision path."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
I = pytest.importorskip("ipmz_amd")
torch = pytest.importorskip("torch")

CHAIN8, ROWS_CHAIN = 2048, 4096  # kernels.h IPMZ_DEBUG_CHAIN8 / IPMZ_DEBUG_ROWS_CHAIN
MODES = [0, CHAIN8, ROWS_CHAIN]


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
        ctx.sync()
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
