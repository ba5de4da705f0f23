"""Object lifetimes at the boundary: a Context destroyed before the solvers
created on it (include/ipmz.h ipmz_ctx_destroy).  The reference's Optimizer
owns its data and settings by value (Optimizer.h:15-20), so its adapters must
survive any destruction order a host language produces -- a garbage
collector finalizing a Context and an Optimizer in one cycle may run either
finalizer first.  Round 5 found exactly that crash in the -m gpu suite
(ipmz_qp_destroy dereferenced a freed context); these tests pin the fix:
the context is only marked, its solvers keep stepping (bitwise as on a
live context), and it is freed with the last of them -- also when two
threads destroy its last solvers at once."""
import ctypes
import gc
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
I = pytest.importorskip("ipmz_amd")
torch = pytest.importorskip("torch")

n_, m_, p_ = 64, 16, 8


def _trace(o, steps, batch=False):
    out = []
    for _ in range(steps):
        o.step()
        out.append(o.batch_scalars().copy() if batch else (o.vars(), o.dir()))
    return out


def _same(a, b):
    for x, y in zip(a, b):
        if isinstance(x, tuple):
            assert all(np.array_equal(u, v) for u, v in zip(x, y))
        else:
            assert np.array_equal(x, y)


def test_solvers_step_after_context_destroyed():
    ref_ctx = I.Context(0)
    ro = I.Optimizer(n_, m_, p_, ref_ctx)
    ro.generate(11)
    rb = I.Batch(n_, m_, p_, 8, ref_ctx)
    rb.generate(100)
    ref_o, ref_b = _trace(ro, 5), _trace(rb, 5, True)
    ro.close(), rb.close(), ref_ctx.close()

    ctx = I.Context(0)
    o = I.Optimizer(n_, m_, p_, ctx)
    o.generate(11)
    b = I.Batch(n_, m_, p_, 8, ctx)
    b.generate(100)
    ctx.close()  # marked only: o and b still use it
    _same(_trace(o, 5), ref_o)
    o.close()  # one user left
    _same(_trace(b, 5, True), ref_b)
    b.close()  # the last user: the context is freed here


def test_context_destroyed_while_on_external_stream():
    """The context runs on torch's stream; destroyed while its solvers live,
    it drains that stream and moves them to its own stream (so its late
    free never touches the caller's stream)."""
    ctx = I.Context(0)
    s = torch.cuda.Stream()
    ctx.set_stream(s.cuda_stream)
    o = I.Optimizer(n_, m_, p_, ctx)
    o.generate(5)
    o.step()
    ctx.close()
    del s
    torch.cuda.synchronize()
    for _ in range(3):
        o.step()
    assert np.isfinite(o.vars()).all()
    o.close()


def test_no_solver_on_a_destroyed_context_c_abi():
    """Through the C ABI: a solver cannot be created on a marked context
    (IPMZ_ERR_STATE), while the one that keeps it alive still steps."""
    lib = I.lib
    h = ctypes.c_void_p()
    assert lib.ipmz_ctx_create(ctypes.byref(h), 0) == 0
    cfg = I._QPConfig(n_, m_, p_, 1e-4, 0, 0, 0, 0)
    q = ctypes.c_void_p()
    assert lib.ipmz_qp_create(h, ctypes.byref(cfg), ctypes.byref(q)) == 0
    assert lib.ipmz_qp_generate(q, 3) == 0
    assert lib.ipmz_ctx_destroy(h) == 0
    assert lib.ipmz_ctx_destroy(h) == 0  # idempotent while marked
    q2 = ctypes.c_void_p()
    assert lib.ipmz_qp_create(h, ctypes.byref(cfg), ctypes.byref(q2)) == -5
    assert not q2.value
    for _ in range(3):
        assert lib.ipmz_qp_step(q, 0) == 0
    assert lib.ipmz_qp_destroy(q) == 0  # frees the context


def test_gc_cycle_finalizes_in_either_order():
    """Context and Optimizer in one reference cycle, left to the collector
    (the round-5 crash), many times over."""
    gc.collect()
    for i in range(40):
        ctx = I.Context(0)
        o = I.Optimizer(n_, m_, p_, ctx) if i % 2 else I.Batch(n_, m_, p_, 4, ctx)
        o.generate(i)
        o.step()
        ctx.cycle = o  # o.ctx -> ctx -> o
        del ctx, o
        gc.collect()
    torch.cuda.synchronize()


def test_concurrent_destroy_of_last_solvers():
    """Two threads destroy the last two solvers of a marked context at once
    (ctypes releases the GIL around each call): exactly one of them frees
    it, none crashes."""
    lib = I.lib
    cfg = I._QPConfig(n_, m_, p_, 1e-4, 0, 0, 0, 0)
    for _ in range(30):
        h = ctypes.c_void_p()
        assert lib.ipmz_ctx_create(ctypes.byref(h), 0) == 0
        qs = []
        for k in range(2):
            q = ctypes.c_void_p()
            assert lib.ipmz_qp_create(h, ctypes.byref(cfg), ctypes.byref(q)) == 0
            assert lib.ipmz_qp_generate(q, k) == 0
            qs.append(q)
        assert lib.ipmz_ctx_destroy(h) == 0
        go = threading.Barrier(2)
        rcs = []

        def kill(q):
            go.wait()
            rcs.append(lib.ipmz_qp_destroy(q))

        ts = [threading.Thread(target=kill, args=(q,)) for q in qs]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert rcs == [0, 0]
