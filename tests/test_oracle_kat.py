"""The reference's Evaluation_test.cpp:107-173 known answers through the CPU
oracle's evaluation of an iterate (the checker the GPU path is compared to;
tests/test_gpu_evaluation_kat.py runs the same values through the device)."""
import numpy as np

import oracle

A = np.array([[1.0, 2.0, 3.0], [4.0, 5.0, 6.0], [7.0, 8.0, 9.0]])
Q = np.array([[1.0, 2.0, 3.0], [2.0, 4.0, 5.0], [3.0, 5.0, 6.0]])
X = np.array([1.0, 2.0, 3.0])
Y = np.array([4.0, 5.0, 6.0])


def _qp(Qm, c):
    return dict(n=3, m=3, p=0, Q=Qm, c=c, A=A, lA=-100.0 * np.ones(3), uA=100.0 * np.ones(3),
                C=np.zeros((0, 3)), d=np.zeros(0), lx=-10.0 * np.ones(3), ux=10.0 * np.ones(3))


def _evaluate(Qm, c, lam_A=None):
    o = oracle.OracleQP(_qp(Qm, c))
    v = {s: np.zeros(oracle.slot_size(s, 3, 3, 0)) for s in o.order}
    v["x"] = X.copy()
    if lam_A is not None:
        v["lambda_A"] = np.asarray(lam_A, dtype=np.float64)
    for s in ("g", "h", "y", "z"):
        v[s] = np.ones(3)
    o.set_vars(np.concatenate([v[s] for s in o.order]))
    r = o.split(-o.rhs(0.0))  # r_v = -rhs_v
    return o.objective(), r


def test_oracle_evaluation_known_answers():
    f, r = _evaluate(Q, np.zeros(3))
    assert r["lambda_A"].tolist() == [14.0, 32.0, 50.0]  # A x
    assert r["x"].tolist() == [14.0, 25.0, 31.0]  # Q x
    assert 2.0 * f == 157.0  # x^T Q x
    f, _ = _evaluate(np.zeros((3, 3)), Y)
    assert f == 32.0  # x^T y
    _, r = _evaluate(np.zeros((3, 3)), np.zeros(3), X)
    assert r["x"].tolist() == [30.0, 36.0, 42.0]  # A^T x
    f, _ = _evaluate(Q, 2.5 * Y)
    assert f == 158.5  # 0.5 x^T Q x + c y^T x
