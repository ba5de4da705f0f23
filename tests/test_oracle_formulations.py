"""InequalityHandling::NaiveSlacks and EqualityHandling::SlackedSlacks in
the CPU oracle (§8f row f4): the formulations against the reference's own
formulas (tests/golden/formulations.txt) and for self-consistency (the
Newton direction solves the Newton system; the optimum is the SlackedSlacks
one).  Both are also pinned to the reference's Newton iterations
(tests/test_oracle_golden.py "naive", "naivereg", "eqss"), made by a harness
that expands the zero (lambda_g, lambda_h) / (lambda_A, lambda_C) block the
reference's evaluator asserts on (Evaluation.cpp:57-60)."""
import os

import numpy as np

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _section(title):
    txt = open(os.path.join(GOLDEN, "formulations.txt")).read()
    i = txt.index(title)
    j = txt.find("\n=== ", i + 1)
    return txt[i:j if j > 0 else len(txt)]


def test_naive_slacks_formulation_is_the_references():
    sec = _section("=== inequality_handling=NaiveSlacks equalities=none inequalities=Both")
    newton = sec.split("-- shorthand definitions")[0]
    assert "variables: [x] [\\lambda_{g}] [\\lambda_{h}] [\\lambda_{y}] [\\lambda_{z}] [g] [h] [y] [z]" in newton
    aug = sec[sec.index("-- augmented system"):]
    assert "variables: [x] [\\lambda_{g}] [\\lambda_{h}]" in aug
    assert "| -A | -(\\Lambda_{g}^{-1} * G) | 0" in aug and "| A | 0 | -(\\Lambda_{h}^{-1} * H)" in aug
    assert "((\\Lambda_{g}^{-1} * r_{g}) - r_{\\lambda_{g}})" in aug
    assert "r_{\\lambda_{g}} := (l_A + g - (A * x))" in sec
    assert "r_{\\lambda_{h}} := (h + (A * x) - u_A)" in sec
    assert "(A^T * (\\lambda_{h} - \\lambda_{g}))" in sec
    assert "\\Delta g := -(\\Lambda_{g}^{-1} * (r_{g} + (G * \\Delta \\lambda_{g})))" in sec


def test_naive_slacks_layout_and_kkt():
    n, m, p = 24, 8, 5
    form = oracle.Form(naive=True)
    o = oracle.OracleQP(oracle.gen_qp(n, m, p, 3), form=form)
    assert o.order == ["x", "lambda_g", "lambda_h", "lambda_C", "p", "lambda_y", "lambda_z", "g", "h", "y", "z"]
    assert o.N == n + 2 * m + p
    K = o.kkt()
    A = o.qp["A"]
    assert np.array_equal(K[n:n + m, :n], -A) and np.array_equal(K[n + m:n + 2 * m, :n], A)
    assert not K[n + m:n + 2 * m, n:n + m].any()  # the zero (lambda_h, lambda_g) block
    assert np.array_equal(np.diag(K)[n:n + 2 * m], -np.ones(2 * m))  # -(L^{-1} G) at g = lambda = 1


def test_naive_slacks_direction_solves_the_newton_system():
    # the augmented solve + back-substitution reproduce every linearised row
    n, m, p = 32, 10, 4
    o = oracle.OracleQP(oracle.gen_qp(n, m, p, 11), form=oracle.Form(naive=True))
    v = o.split(o.vars())
    o.iterate()
    d = o.split(o.daff())
    qp = o.qp
    # primal rows: -A dx + dg = -r_lg, A dx + dh = -r_lh, with r at mu = 0
    Ax = qp["A"] @ v["x"]
    r_lg = (qp["lA"] + v["g"]) - Ax
    r_lh = (v["h"] + Ax) - qp["uA"]
    assert np.abs(-qp["A"] @ d["x"] + d["g"] + r_lg).max() < 1e-10
    assert np.abs(qp["A"] @ d["x"] + d["h"] + r_lh).max() < 1e-10
    # complementarity: lambda_g dg + G dlambda_g = -(G lambda_g)
    assert np.abs(v["lambda_g"] * d["g"] + v["g"] * d["lambda_g"] + v["g"] * v["lambda_g"]).max() < 1e-10


def test_naive_slacks_reaches_the_slacked_slacks_optimum():
    n, m, p = 48, 16, 6
    out = {}
    for naive in (False, True):
        o = oracle.OracleQP(oracle.gen_qp(n, m, p, 7), form=oracle.Form(naive=naive))
        for it in range(60):
            done, rec = o.iterate()
            if done:
                break
        assert done == 1
        out[naive] = o.split(o.vars())["x"]
    assert np.abs(out[True] - out[False]).max() < 1e-8



def _rename_a_to_c(t):
    """The lambda_A / s / g / h block's text with the lambda_C / t / v / w names."""
    import re
    for a, b in ((r"\lambda_{A}", r"\lambda_{C}"), (r"\lambda_{g}", r"\lambda_{v}"), (r"\lambda_{h}", r"\lambda_{w}"),
                 (r"\Lambda_{g}", r"\Lambda_{v}"), (r"\Lambda_{h}", r"\Lambda_{w}"), ("r_{s}", "r_{t}"),
                 ("r_{g}", "r_{v}"), ("r_{h}", "r_{w}"), ("e_{A}", "e_{C}"), ("l_A", "d"), ("u_A", "d")):
        t = t.replace(a, b)
    t = re.sub(r"\bG\b", "V", t)
    t = re.sub(r"\bH\b", "W", t)
    t = re.sub(r"\bA\b", "C", t)
    t = re.sub(r"(?<![_{\\])\bs\b", "t", t)
    t = re.sub(r"(?<![_{\\])\bg\b", "v", t)
    t = re.sub(r"(?<![_{\\])\bh\b", "w", t)
    return t


def test_equality_slacked_slacks_is_the_inequality_block_with_d():
    # EqualityHandling::SlackedSlacks (SymbolicOptimization.cpp:150-161): every
    # lambda_C / t / v / w formula is the lambda_A / s / g / h one renamed, with
    # l_A = u_A = d -- what oracle.eqss_merge and the GPU's [A; C] rows rely on
    sec = _section("=== inequality_handling=SlackedSlacks equalities=SlackedSlacks inequalities=Both")
    defs = {}
    for ln in sec.splitlines():
        if " := " in ln:
            k, v = ln.strip().split(" := ")
            defs.setdefault(k, v)
    pairs = [(r"r_{\lambda_{A}}", r"r_{\lambda_{C}}"), ("r_{s}", "r_{t}"), (r"r_{\lambda_{g}}", r"r_{\lambda_{v}}"),
             (r"r_{\lambda_{h}}", r"r_{\lambda_{w}}"), ("r_{g}", "r_{v}"), ("r_{h}", "r_{w}"),
             (r"\Delta s", r"\Delta t"), (r"\Delta g", r"\Delta v"), (r"\Delta h", r"\Delta w"),
             (r"\Delta \lambda_{g}", r"\Delta \lambda_{v}"), (r"\Delta \lambda_{h}", r"\Delta \lambda_{w}")]
    for a, c in pairs:
        got, want = defs[c], _rename_a_to_c(defs[a])
        if got != want:  # (v + d - t) vs (l_A + g - s): the same sum with the operands commuted
            assert sorted(got.strip("()").replace(" - ", " + -").split(" + ")) == \
                sorted(want.strip("()").replace(" - ", " + -").split(" + ")), (c, got, want)
    aug = sec[sec.index("-- augmented system"):sec.index("-- normal equations")]
    rows = [ln.strip().strip("|").split(" | ") for ln in aug.splitlines() if ln.strip().startswith("|")]
    assert rows[2][2].strip() == _rename_a_to_c(rows[1][1].strip())
    assert rows[1][2].strip() == "0" and rows[2][1].strip() == "0"
    rhs = [ln.strip() for ln in aug.split("rhs:")[1].split("delta_definitions:")[0].splitlines() if ln.strip()]
    assert rhs[2] == _rename_a_to_c(rhs[1])
