"""The blocked factors are deterministic: which workgroup of which launch runs a
role never changes the arithmetic (panel.hip), so repeated factorizations of
one matrix must agree bit for bit.  A missing ordering between the
factor's streams or a stale hand-off shows up here as run-to-run differences
(it did: the mixed-precision factor's rows stream once started before the
fp32 conversion on the chain stream had finished).

fp64 (LinearSolvers::ldlt_decomposition, LinearSolvers.cpp:14-42, blocked)
and the fp32 factor of the mixed-precision path, on the look-ahead schedule
(>= 3 outer panels: the factor forks onto three streams)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
I = pytest.importorskip("ipmz_amd")
torch = pytest.importorskip("torch")
REPS = 4


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


@pytest.mark.parametrize("N", [1408, 4096])
def test_fp64_factor_bitwise_repeatable(ctx, N):
    K = _qd(N, N)
    wsb = ctx.workspace_bytes(N)
    ws = torch.zeros(wsb // 8 + 1, dtype=torch.float64, device="cuda")
    D = torch.zeros(N, dtype=torch.float64, device="cuda")
    out = []
    for _ in range(REPS):
        Kf = K.clone()
        assert ctx.ldlt_factor(N, Kf.data_ptr(), N, D.data_ptr(), ws.data_ptr(), wsb) == 0
        torch.cuda.synchronize()
        out.append((torch.tril(Kf, -1).cpu().numpy(), D.cpu().numpy()))
    for r in range(1, REPS):
        assert np.array_equal(out[r][0], out[0][0]) and np.array_equal(out[r][1], out[0][1]), r


@pytest.mark.parametrize("N", [1408, 4096])
def test_fp32_mixed_factor_bitwise_repeatable(ctx, N):
    K = _qd(N, N + 1)
    wsb = ctx.mixed_workspace_bytes(N)
    ws = torch.zeros(wsb // 4 + 64, dtype=torch.float32, device="cuda")
    ld32 = (N + 63) // 64 * 64
    doff = ((N * ld32 * 4 + 255) // 256 * 256) // 4  # D32 follows K32 (mixed_ws_carve)
    out = []
    for _ in range(REPS):
        ws.zero_()
        assert ctx.mixed_factor(N, K.data_ptr(), N, ws.data_ptr(), wsb) == 0
        torch.cuda.synchronize()
        L = torch.tril(ws[:N * ld32].view(N, ld32)[:, :N], -1)
        out.append((L.cpu().numpy(), ws[doff:doff + N].cpu().numpy()))
    for r in range(1, REPS):
        assert np.isfinite(out[r][0]).all()
        assert np.array_equal(out[r][0], out[0][0]) and np.array_equal(out[r][1], out[0][1]), r


@pytest.mark.parametrize("N,reps", [(2560, 300), (4096, 200)])
def test_fp64_early_chain_factor_run_to_run_long(ctx, N, reps):
    """The early-chain panel path (each chain launch starts beside the
    previous panel's rows launch, gated by RDONE flags; 384-wide panels at
    C2's N = 2560, the last panels of N = 4096) over hundreds of factors in
    one process, bitwise against the first: the cross-launch gates are the
    kind of race a 4-factor check cannot see (the C4 factor's was once in
    ~360 factors, test_c4_eager_steps_run_to_run_bitwise)."""
    K = _qd(N, N + 2)
    wsb = ctx.workspace_bytes(N)
    ws = torch.zeros(wsb // 8 + 1, dtype=torch.float64, device="cuda")
    D = torch.zeros(N, dtype=torch.float64, device="cuda")
    Kf = torch.empty_like(K)
    first = None
    bad = []
    for r in range(reps):
        Kf.copy_(K)
        assert ctx.ldlt_factor(N, Kf.data_ptr(), N, D.data_ptr(), ws.data_ptr(), wsb) == 0
        out = (torch.tril(Kf, -1), D.clone())
        if first is None:
            first = out
            assert torch.isfinite(first[0]).all() and torch.isfinite(first[1]).all()
        elif not (torch.equal(out[0], first[0]) and torch.equal(out[1], first[1])):
            bad.append(r)
    ctx.sync()
    assert not bad, bad[:8]


def test_c2_normal_steps_run_to_run_long(ctx):
    """Two C2 solvers (n = 2048, m = 512, normal equations) from the same
    seed, 200 eager Newton steps each, restarting converged ones: iterates
    and directions bitwise equal after every step."""
    g = [I.Optimizer(2048, 512, 0, ctx) for _ in range(2)]
    for o in g:
        o.generate(1234)
        o.set_reduction(I.REDUCTION_NORMAL)
    for it in range(200):
        for o in g:
            o.step(I.STEP_RESTART_IF_CONVERGED)
        v0, v1 = g[0].vars(), g[1].vars()
        assert np.array_equal(v0, v1), it
        assert np.array_equal(g[0].dir(), g[1].dir()), it
    for o in g:
        o.close()
