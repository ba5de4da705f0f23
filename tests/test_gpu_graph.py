"""HIP-graph capture of whole Newton steps whose factorization forks onto the
look-ahead streams (>= 3 outer panels).  The production path enqueues such
steps eagerly (graph replay of the forked step measured slower,
tools/graph_ab.py); debug bit INJECT_GRAPH_FORKS makes IPMZ_STEP_GRAPH capture
them.  The capture must end (the HIP runtime torch bundles used to recurse
without end inside hipStreamEndCapture on the look-ahead's cross-stream
waits: ldlt.hip stream_record / stream_wait) and the replayed step must equal
the eager step bit for bit: the same kernels, the same order of every
dependent pair -- one Newton step of Optimizer::solve (Optimizer.cpp:127-219)
from the same iterate."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
I = pytest.importorskip("ipmz_amd")
torch = pytest.importorskip("torch")


@pytest.fixture(autouse=True)
def graph_forks():
    I.debug_inject(I.INJECT_GRAPH_FORKS)
    yield
    I.debug_inject(0)


def _pair(ctx, n, m, p, mode):
    qs = []
    for _ in range(2):
        q = I.Optimizer(n, m, p, ctx)
        q.generate(77)
        if mode == "normal":
            q.set_reduction(I.REDUCTION_NORMAL)
        if mode == "mixed":
            q.set_mixed_precision(True, 1e-12, 20)
        qs.append(q)
    return qs


@pytest.mark.parametrize("n,m,p,mode,torch_stream", [
    (1024, 256, 128, "augmented", False),   # N = 1408: 6 outer panels of 256
    (1024, 256, 128, "augmented", True),    # on torch's (legacy default) stream: captured on the context's own
    (2048, 512, 0, "normal", False),        # C2's shape: the pipelined normal-equations factor, 7 panels of 384
    (1536, 0, 0, "mixed", False),           # fp32 factor + fp64 refinement, 6 panels
    (5120, 0, 0, "mixed", False),           # 10 panels of 512: the 128 x 128 f32 trailing tiles too
])
def test_captured_forked_step_equals_eager(n, m, p, mode, torch_stream):
    ctx = I.Context(0, stream=torch.cuda.current_stream().cuda_stream) if torch_stream else I.Context(0)
    try:
        N = n + m + p
        nbo = ctx.blocking(N)[0]
        assert (N + nbo - 1) // nbo >= 3  # the factor forks
        eager, graph = _pair(ctx, n, m, p, mode)
        flags = I.STEP_RESTART_IF_CONVERGED
        for it in range(4):
            eager.step(flags)
            graph.step(flags | I.STEP_GRAPH)
            ctx.sync()
            assert graph.last_step_graph() == 1 and eager.last_step_graph() == 0
            for which in (1, 2):  # affine and corrector directions
                assert np.array_equal(eager._state(which), graph._state(which)), (it, which)
            assert np.array_equal(eager.vars(), graph.vars()), it
        eager.close()
        graph.close()
    finally:
        ctx.close()


@pytest.mark.parametrize("n,m,p,mode", [
    (1024, 256, 128, "augmented"),  # N = 1408, 6 outer panels: the forked factor
    (1536, 0, 0, "mixed"),          # the mixed solve enqueues every refinement pass inside a capture
])
def test_step_inside_callers_torch_graph_capture(n, m, p, mode):
    """A caller that captures step() itself (torch.cuda.graph on the
    context's stream): the step goes into the caller's capture on that
    stream -- no hop to the context's own stream, no host wait -- and each
    replay equals an eager step bit for bit."""
    s = torch.cuda.Stream()
    ctx = I.Context(0, stream=s.cuda_stream)
    try:
        eager, graph = _pair(ctx, n, m, p, mode)
        flags = I.STEP_RESTART_IF_CONVERGED
        eager.step(flags)  # first steps eager: workspaces exist before the capture
        graph.step(flags)
        ctx.sync()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            graph.step(flags)
        for it in range(3):
            eager.step(flags)
            with torch.cuda.stream(s):
                g.replay()
            s.synchronize()
            ctx.sync()
            for which in (1, 2):
                assert np.array_equal(eager._state(which), graph._state(which)), (it, which)
            assert np.array_equal(eager.vars(), graph.vars()), it
        eager.close()
        graph.close()
    finally:
        ctx.close()
