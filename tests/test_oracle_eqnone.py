"""EqualityHandling::None in the CPU oracle (§8f row f3).

The reference routes a KKT matrix with a zero diagonal block to
Optimizer::solve_indefinite_ (Optimizer.cpp:63-75), which is ASSERT(false):
it has no end-to-end numeric path for this formulation.  Parity is pinned at
the component level:
  * the formulation (augmented lhs/rhs, shorthand and delta definitions) is
    the reference's own symbolic output (tests/golden/formulations.txt);
  * the factor is the reference's symmetric_indefinite_factorization /
    overwriting_solve_bunch_kaufman, restated bitwise
    (tests/test_oracle_golden.py, bk_* fixtures);
  * the end-to-end Newton iteration is the oracle's restatement (parity
    unpinned end-to-end: the reference asserts)."""
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _section(title):
    txt = open(os.path.join(GOLDEN, "formulations.txt")).read()
    i = txt.index(title)
    j = txt.find("\n=== ", i + 1)
    return txt[i:j if j > 0 else len(txt)]


def test_formulation_is_the_references():
    sec = _section("=== inequality_handling=SlackedSlacks equalities=None inequalities=Both")
    aug = sec[sec.index("-- augmented system"):sec.index("-- normal equations")]
    # no p variable, zero (lambda_C, lambda_C) block, rhs -r_lambda_C
    assert "variables: [x] [\\lambda_{A}] [\\lambda_{C}]" in aug
    assert "| C | 0 | 0" in aug
    assert "    -r_{\\lambda_{C}}" in aug
    assert "r_{\\lambda_{C}} := ((C * x) - d)" in sec
    assert "[p]" not in sec.split("-- shorthand definitions")[0]


def test_kkt_and_state_layout():
    n, m, p = 24, 8, 5
    qp = oracle.gen_qp(n, m, p, 5)
    o = oracle.OracleQP(qp, eq_none=True)
    r = oracle.OracleQP(qp)
    assert "p" not in o.order and o.L == r.L - p
    Kn, Kr = o.kkt(), r.kkt()
    N = n + m + p
    assert np.all(Kn[n + m:, n + m:] == 0.0)
    Kr[n + m:, n + m:] = 0.0
    assert np.array_equal(Kn, Kr)
    b = o.rhs()
    res = o.split(o._get("ipmzo_get_vars"))  # iterate layout matches the order
    assert len(res["lambda_C"]) == p and len(b) == N


@pytest.mark.parametrize("n,m,p,seed", [(40, 10, 6, 3), (64, 16, 8, 1234), (30, 0, 4, 9)])
def test_newton_direction_solves_the_system(n, m, p, seed):
    qp = oracle.gen_qp(n, m, p, seed)
    o = oracle.OracleQP(qp, eq_none=True)
    K, b = o.kkt(), o.rhs(0.0)
    o.iterate()
    d = o.split(o.daff())
    sol = np.concatenate([d["x"], d.get("lambda_A", np.zeros(0)), d["lambda_C"]])
    # Bunch-Kaufman solve of the indefinite system: residual at rounding level
    assert np.abs(K @ sol - b).max() < 1e-12 * max(1.0, np.abs(b).max())


def test_converges_near_regularization():
    qp = oracle.gen_qp(40, 10, 6, 3)
    out = {}
    for eq_none in (False, True):
        o = oracle.OracleQP(qp, eq_none=eq_none)
        for it in range(100):
            done, rec = o.iterate()
            if done:
                break
        assert done
        out[eq_none] = (it, o.split(o.vars())["x"])
    # same optimum up to the O(delta) regularization perturbation
    assert np.abs(out[True][1] - out[False][1]).max() < 1e-6


def test_penalty_formulation_and_kkt():
    sec = _section("=== inequality_handling=SlackedSlacks equalities=PenaltyFunction inequalities=Both")
    aug = sec[sec.index("-- augmented system"):sec.index("-- normal equations")]
    assert "| C | 0 | -\\mu" in aug and "    -r_{\\lambda_{C}}" in aug
    assert "r_{\\lambda_{C}} := -(d + (\\mu * \\lambda_{C}) - (C * x))" in sec
    n, m, p = 24, 8, 5
    qp = oracle.gen_qp(n, m, p, 5)
    o = oracle.OracleQP(qp, eq_penalty=True)
    K = o.kkt()
    assert np.array_equal(np.diag(K)[n + m:], -np.ones(p))  # environment mu = 1 at the start
    o.iterate()
    d = o.split(o.daff())
    assert "p" not in o.order and len(d["lambda_C"]) == p


def test_penalty_extra_dual_is_the_same_newton_system():
    # Settings::EqualityHandling::PenaltyFunctionWithExtraDual: the reference
    # derives PenaltyFunction's optimality conditions through it
    # (SymbolicOptimization.cpp:364-366), and its symbolic output for both is
    # the same Newton system, shorthand and augmented system -- so
    # IPMZ_EQ_PENALTY_EXTRA_DUAL runs the PenaltyFunction path
    pf = _section("=== inequality_handling=SlackedSlacks equalities=PenaltyFunction inequalities=Both")
    px = _section("=== inequality_handling=SlackedSlacks equalities=PenaltyFunctionWithExtraDual inequalities=Both")
    assert pf.split("\n", 1)[1] == px.split("\n", 1)[1]
