"""Parity at the benchmarked sizes: one Newton step of the HIP path against the
CPU oracle on identical inputs, at BASELINE.json's full C3 and C5 sizes.

The oracle's factor here is ldlt_blocked (oracle/ipmz_oracle.cpp): the
reference's LDL^T (LinearSolvers.cpp:14-42) bit for bit -- pinned in
tests/test_oracle_golden.py -- reorganised so the full-size factor finishes in
seconds on the box's host cores.  Each comparison starts from the same
iterate (Optimizer.cpp:137-217: assembly, factor, predictor and corrector
solves, back-substitution, ratio tests).

Tolerances (written here, BASELINE.json north_star):
  * ||dx_gpu - dx_cpu||_inf < 1e-10 for the affine AND the corrector
    direction;
  * every other Newton block within 1e-9 relative to its own max-norm;
  * alpha_aff, mu_aff, sigma, alpha within 1e-9 relative.
"""
import time

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

I = pytest.importorskip("ipmz_amd")

DX_TOL = 1e-10


@pytest.fixture(scope="module")
def ctx():
    return I.Context(0)


def _check_step(o, g, label):
    errs = {}
    for which, (go, oo) in enumerate(((g.daff(), o.daff()), (g.dir(), o.dir()))):
        sg, so = o.split(go), o.split(oo)
        for s in o.order:
            scale = max(1.0, np.abs(so[s]).max())
            err = np.abs(sg[s] - so[s]).max()
            errs[(which, s)] = err
            assert err < 1e-9 * scale, (label, which, s, err, scale)
        dx = np.abs(sg["x"] - so["x"]).max()
        print(f"{label}: {'affine' if which == 0 else 'corrector'} |dx_gpu - dx_cpu|_inf = {dx:.3e}", flush=True)
        assert dx < DX_TOL, (label, which, dx)
    return errs


def _check_scalars(g, rec, label):
    s = g.scalars()
    for k in ("alpha_aff", "mu_aff", "sigma", "alpha"):
        assert abs(s[k] - rec[k]) <= 1e-9 * max(1.0, abs(rec[k])), (label, k, s[k], rec[k])


def test_c3_newton_steps_vs_oracle(ctx):
    """C3 (BASELINE.json configs[2]): n=8192, m=2048, p=1024, N=11264, seed
    1234 -- at the initial iterate and at the GPU's iterate after 4 steps."""
    n, m, p, seed = 8192, 2048, 1024, 1234
    t0 = time.time()
    qp = oracle.gen_qp(n, m, p, seed)
    o = oracle.OracleQP(qp)
    g = I.Optimizer(n, m, p, ctx)
    g.generate(seed)
    assert np.array_equal(g.vars(), o.vars())  # generator + build_environment: bitwise
    for label, warm in (("C3 iterate 0", 0), ("C3 iterate 4", 4)):
        for _ in range(warm):
            g.step()
        if warm:
            o.set_vars(g.vars())
        s0 = g.scalars()
        g.step()
        done, rec = o.iterate()
        assert done == 0
        for k in ("f", "res", "mu"):
            assert abs(s0[k] - rec[k]) <= 1e-12 * max(1.0, abs(rec[k])), (label, k, s0[k], rec[k])
        _check_scalars(g, rec, label)
        _check_step(o, g, label)
        g.set_vars(o.vars())  # both continue from the oracle's updated iterate
        print(f"{label}: done at {time.time() - t0:.1f} s", flush=True)


def test_c5_mixed_newton_step_vs_oracle(ctx):
    """C5 (BASELINE.json configs[4]): n=16384 box-only, fp32 factor of the
    scaled KKT matrix + fp64 iterative refinement at tol 1e-14, against the
    oracle's fp64 reference-order factor."""
    n, seed = 16384, 1234
    qp = oracle.gen_qp(n, 0, 0, seed)
    o = oracle.OracleQP(qp)
    g = I.Optimizer(n, 0, 0, ctx)
    g.generate(seed)
    g.set_mixed_precision(True, 1e-14, 30)
    assert np.array_equal(g.vars(), o.vars())
    g.step()
    done, rec = o.iterate()
    assert done == 0
    _check_scalars(g, rec, "C5 iterate 0")
    _check_step(o, g, "C5 iterate 0")
    s = g.scalars()
    print(f"C5: refinement ratio {s['ir_ratio_aff']:.2e} / {s['ir_ratio']:.2e} after "
          f"{s['ir_iters_aff']:.0f} / {s['ir_iters']:.0f} corrections", flush=True)


def test_c5_mixed_bench_setting_vs_oracle(ctx):
    """C5 at the setting bench.py times (refinement tolerance 1e-12, at most
    20 corrections, bench.py --ir-tol default): the same parity bar as the
    fp64 path, ||dx_gpu - dx_cpu||_inf < 1e-10, at iterate 0 and at the
    GPU's iterate after 3 steps."""
    n, seed = 16384, 1234
    qp = oracle.gen_qp(n, 0, 0, seed)
    o = oracle.OracleQP(qp)
    g = I.Optimizer(n, 0, 0, ctx)
    g.generate(seed)
    g.set_mixed_precision(True, 1e-12, 20)
    assert np.array_equal(g.vars(), o.vars())
    for label, warm in (("C5@1e-12 iterate 0", 0), ("C5@1e-12 iterate 3", 3)):
        for _ in range(warm):
            g.step()
        if warm:
            o.set_vars(g.vars())
        g.step()
        done, rec = o.iterate()
        assert done == 0
        _check_scalars(g, rec, label)
        _check_step(o, g, label)
        s = g.scalars()
        assert s["ir_ratio"] <= 1e-12 and s["ir_ratio_aff"] <= 1e-12, s
        print(f"{label}: refinement ratio {s['ir_ratio_aff']:.2e} / {s['ir_ratio']:.2e} after "
              f"{s['ir_iters_aff']:.0f} / {s['ir_iters']:.0f} corrections", flush=True)
        g.set_vars(o.vars())


def test_c2_normal_newton_steps_vs_oracle(ctx):
    """C2 (BASELINE.json configs[1]): n=2048, m=512, the normal-equations
    reduction (Cholesky of H, TRSM, SYRK, Cholesky of S as one pipelined
    factor, 384-wide outer panels at this size) against the oracle's
    augmented reference-order LDL^T from the same iterate -- the Newton
    directions are the same system's solution (Optimizer.cpp:137-217,
    SymbolicOptimization.cpp:465-478), at iterate 0 and after 4 steps."""
    n, m, p, seed = 2048, 512, 0, 1234
    qp = oracle.gen_qp(n, m, p, seed)
    o = oracle.OracleQP(qp)
    g = I.Optimizer(n, m, p, ctx)
    g.generate(seed)
    g.set_reduction(I.REDUCTION_NORMAL)
    assert ctx.blocking(n + m)[0] == 384  # the blocking bench.py's C2 line runs
    assert np.array_equal(g.vars(), o.vars())
    for label, warm in (("C2 iterate 0", 0), ("C2 iterate 4", 4)):
        for _ in range(warm):
            g.step()
        if warm:
            o.set_vars(g.vars())
        g.step()
        done, rec = o.iterate()
        assert done == 0
        _check_scalars(g, rec, label)
        _check_step(o, g, label)
        g.set_vars(o.vars())
