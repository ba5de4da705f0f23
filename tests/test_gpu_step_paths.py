"""Round-3 production-path switches of the Newton step, each against the
path it replaced on the same iterate (one Newton step of Optimizer::solve,
Optimizer.cpp:127-219):

* the fp32 trailing and strip updates (mixed precision, C5) on the
  32 x 32 x 2 f32 MFMA kernel (gemm32.h) vs the gemm.h engine's fp32
  instance (debug bit 128): the same directions to refinement tolerance, and
  two runs bitwise equal (every element of C written by one launch, in a
  fixed k order);
* the eager refinement loop that stops on a host-mapped stop test vs all
  max_refine + 1 passes enqueued (debug bit 512): bitwise equal (the passes
  after convergence return at once);
* the forked step on a caller-made stream (torch's) -- run on the context's
  own stream, host-joined -- vs the context's own stream: bitwise equal.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
I = pytest.importorskip("ipmz_amd")
torch = pytest.importorskip("torch")

DEBUG_F32_ENGINE, DEBUG_IR_FULL = 128, 512


@pytest.fixture(autouse=True)
def clear_debug():
    yield
    I.debug_inject(0)


def _run(ctx, n, m, p, steps, mixed, mask=0):
    I.debug_inject(mask)
    q = I.Optimizer(n, m, p, ctx)
    q.generate(321)
    if mixed:
        q.set_mixed_precision(True, 1e-12, 20)
    out = []
    for _ in range(steps):
        q.step(I.STEP_RESTART_IF_CONVERGED)
        ctx.sync()
        out.append((q.daff(), q.dir(), q.vars(), q.scalars()))
    q.close()
    I.debug_inject(0)
    return out


def test_f32_mfma_kernel_vs_gemm_engine_and_determinism():
    ctx = I.Context(0)
    try:
        n = 6144  # N = 6144, nbo 512: trailing orders 5120 .. 512 (both tile sizes), strips
        mf = _run(ctx, n, 0, 0, 2, True)
        mf2 = _run(ctx, n, 0, 0, 2, True)
        eng = _run(ctx, n, 0, 0, 2, True, DEBUG_F32_ENGINE)
        for (a1, d1, v1, s1), (a2, d2, v2, _), (a3, d3, v3, s3) in zip(mf, mf2, eng):
            assert np.array_equal(a1, a2) and np.array_equal(d1, d2) and np.array_equal(v1, v2)
            assert s1["ir_ratio_aff"] <= 1e-12 and s1["ir_ratio"] <= 1e-12
            assert s3["ir_ratio_aff"] <= 1e-12 and s3["ir_ratio"] <= 1e-12
            for x, y in ((a1, a3), (d1, d3), (v1, v3)):
                assert np.max(np.abs(x - y)) <= 1e-9 * max(1.0, np.max(np.abs(y)))
    finally:
        ctx.close()


def test_host_stop_test_equals_full_refinement_loop():
    ctx = I.Context(0)
    try:
        stop = _run(ctx, 2048, 0, 0, 3, True)
        full = _run(ctx, 2048, 0, 0, 3, True, DEBUG_IR_FULL)
        for (a1, d1, v1, s1), (a2, d2, v2, s2) in zip(stop, full):
            assert np.array_equal(a1, a2) and np.array_equal(d1, d2) and np.array_equal(v1, v2)
            assert s1["ir_iters_aff"] == s2["ir_iters_aff"] and s1["ir_iters"] == s2["ir_iters"]
    finally:
        ctx.close()


@pytest.mark.parametrize("mixed", [False, True])
def test_forked_step_on_torch_stream_equals_own_stream(mixed):
    own = I.Context(0)
    ext = I.Context(0, stream=torch.cuda.current_stream().cuda_stream)
    try:
        n, m, p = (1536, 0, 0) if mixed else (1024, 256, 128)
        assert (n + m + p + ext.blocking(n + m + p)[0] - 1) // ext.blocking(n + m + p)[0] >= 3  # forks
        a = _run(own, n, m, p, 3, mixed)
        b = _run(ext, n, m, p, 3, mixed)
        for (a1, d1, v1, _), (a2, d2, v2, _) in zip(a, b):
            assert np.array_equal(a1, a2) and np.array_equal(d1, d2) and np.array_equal(v1, v2)
        # stream order: the state read on the caller's stream right after
        # step(), with no synchronisation in between, is the step's result
        q = I.Optimizer(n, m, p, ext)
        q.generate(321)
        if mixed:
            q.set_mixed_precision(True, 1e-12, 20)
        q.step(I.STEP_RESTART_IF_CONVERGED)
        assert np.array_equal(q.vars(), a[0][2])
        q.close()
    finally:
        own.close()
        ext.close()
