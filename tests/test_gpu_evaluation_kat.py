"""The reference's only numeric known-answer tests, restated through the
device kernels that evaluate the same expressions in the Newton step.

/root/reference/test/Evaluation_test.cpp:107-173 evaluates, with
A = [[1,2,3],[4,5,6],[7,8,9]], Q = [[1,2,3],[2,4,5],[3,5,6]], x = [1,2,3],
y = [4,5,6], c = 2.5:
  A x = [14, 32, 50]            (EvaluateMatrices, :118-129)
  A^T (transpose elements)      (:131-140)
  x^T y = 32                    (EvaluateComplexExpressions, :145-150)
  x^T Q x = 157                 (:152-162)
  0.5 x^T Q x + c y^T x = 158.5 (:164-172)
Here they go through the GPU evaluation of an iterate (ipmz_qp_set_state ->
k_residuals / objective, newton.hip): the objective scalar IPMZ_SC_F is
0.5 x'Qx + c'x, the lambda_A residual block is A x - s and the x block is
c + lambda_z + Q x + A^T lambda_A - lambda_y (formulations.txt shorthand
definitions).  Every value is an exact small integer or half-integer in
fp64, so the checks are equalities.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

I = pytest.importorskip("ipmz_amd")

A = np.array([[1.0, 2.0, 3.0], [4.0, 5.0, 6.0], [7.0, 8.0, 9.0]])
Q = np.array([[1.0, 2.0, 3.0], [2.0, 4.0, 5.0], [3.0, 5.0, 6.0]])
X = np.array([1.0, 2.0, 3.0])
Y = np.array([4.0, 5.0, 6.0])
SCALAR_C = 2.5


@pytest.fixture(scope="module")
def ctx():
    return I.Context(0)


def _evaluate(ctx, Qm, c, lam_A=None):
    """Load the 3-variable, 3-row QP, set the iterate (x, s = 0, lambda_A,
    positive slacks 1, other duals 0) and return (f, {slot: residual})."""
    n = m = 3
    data = I.Data(Qm, c, -10.0 * np.ones(n), 10.0 * np.ones(n), A, -100.0 * np.ones(m), 100.0 * np.ones(m))
    opt = I.Optimizer.from_data(data, ctx)
    order = oracle.newton_order(n, m, 0)
    v = {s: np.zeros(oracle.slot_size(s, n, m, 0)) for s in order}
    v["x"] = X.copy()
    if lam_A is not None:
        v["lambda_A"] = np.asarray(lam_A, dtype=np.float64)
    for s in ("g", "h", "y", "z"):
        v[s] = np.ones(oracle.slot_size(s, n, m, 0))
    opt.set_vars(np.concatenate([v[s] for s in order]))
    f = opt.scalars()["f"]
    r = opt.residuals()
    out, off = {}, 0
    for s in order:
        k = oracle.slot_size(s, n, m, 0)
        out[s] = r[off:off + k]
        off += k
    opt.close()
    return f, out


def test_matrix_vector_product(ctx):
    # Evaluation_test.cpp:118-129: A x = [14, 32, 50] (the lambda_A residual A x - s, s = 0)
    _, r = _evaluate(ctx, Q, np.zeros(3))
    assert r["lambda_A"].tolist() == [14.0, 32.0, 50.0]


def test_transpose(ctx):
    # Evaluation_test.cpp:131-140 (A^T[0][1] = 4, A^T[1][2] = 8, A^T[2][0] = 3): with
    # Q = 0, c = 0 the x residual is A^T lambda_A; lambda_A = e_1 picks A^T's column 1
    # = A's row 1, e_2 picks A's row 2 -- A^T[0][1] = 4 and A^T[1][2] = 8 --, e_0 row 0
    for k, row in ((0, A[0]), (1, A[1]), (2, A[2])):
        e = np.zeros(3)
        e[k] = 1.0
        _, r = _evaluate(ctx, np.zeros((3, 3)), np.zeros(3), e)
        assert r["x"].tolist() == row.tolist()
    _, r = _evaluate(ctx, np.zeros((3, 3)), np.zeros(3), X)
    assert r["x"].tolist() == (A.T @ X).tolist() == [30.0, 36.0, 42.0]


def test_dot_product(ctx):
    # Evaluation_test.cpp:145-150: x^T y = 32 (objective with Q = 0, c = y)
    f, _ = _evaluate(ctx, np.zeros((3, 3)), Y)
    assert f == 32.0


def test_quadratic_form(ctx):
    # Evaluation_test.cpp:152-162: x^T Q x = 157 (objective 0.5 x'Qx with c = 0); Q x = [14, 25, 31]
    f, r = _evaluate(ctx, Q, np.zeros(3))
    assert 2.0 * f == 157.0
    assert r["x"].tolist() == [14.0, 25.0, 31.0]


def test_combined_expression(ctx):
    # Evaluation_test.cpp:164-172: 0.5 x^T Q x + c y^T x = 158.5 (c_vec = 2.5 y)
    f, _ = _evaluate(ctx, Q, SCALAR_C * Y)
    assert f == 158.5
