"""Bunch-Kaufman (LinearSolvers.cpp:76-318) on the GPU
against the reference's golden vectors and the CPU oracle.

The factor updates every element with the reference's own expression and
operand order, so F and ipiv are compared BITWISE -- including the fixtures
that force interchanges and 2x2 pivots (bkr*) and the one with two zero
columns that trips the reference's kp = 0 defect (bkz16), and the one whose
first zero column is column 0 (bkz0_16: the reference's 0-based info stays 0,
LinearSolvers.cpp:113-116, so the next zero column still takes kp = k).  The solve's
backward dot products are tree reductions: x within 1e-13 relative.
"""
import numpy as np
import pytest

import oracle
from golden_io import load

pytestmark = pytest.mark.gpu
I = pytest.importorskip("ipmz_amd")
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ctx():
    return I.Context(0)


@pytest.mark.parametrize("N,tag", [(8, "bk8"), (64, "bk64"), (8, "bkr8"), (64, "bkr64"), (200, "bkr200"),
                                   (16, "bkz16"), (16, "bkz0_16")])
def test_bk_golden(ctx, N, tag):
    K = load(f"{tag}_K.bin").reshape(N, N)
    F, ipiv = I.LinearSolvers.symmetric_indefinite_factorization(K, ctx)
    assert np.array_equal(F, load(f"{tag}_F.bin").reshape(N, N))
    assert np.array_equal(ipiv, load(f"{tag}_ipiv.bin").astype(np.int32))
    x = load(f"{tag}_b.bin").copy()
    I.LinearSolvers.overwriting_solve_bunch_kaufman(F, ipiv, x, ctx)
    ref = load(f"{tag}_x.bin")
    if np.isfinite(ref).all():
        assert np.abs(x - ref).max() <= 1e-13 * max(1.0, np.abs(ref).max())
    else:  # the reference's defect divides by zero: the same entries are non-finite
        assert np.array_equal(np.isfinite(x), np.isfinite(ref))


def _indef(N, seed, zeros=0):
    rng = np.random.default_rng(seed)
    K = rng.uniform(-1, 1, (N, N))
    K = np.tril(K) + np.tril(K, -1).T
    K[np.arange(N), np.arange(N)] *= 0.05
    for z in range(zeros):
        K[N // 2 + z, :] = 0
        K[:, N // 2 + z] = 0
    return K


@pytest.mark.parametrize("N", [1, 2, 3, 100, 513, 1500])
def test_bk_vs_oracle_bitwise(ctx, N):
    K = _indef(N, N)
    F, ipiv = I.LinearSolvers.symmetric_indefinite_factorization(K, ctx)
    Fo, po, _ = oracle.bk_factor(K)
    assert np.array_equal(ipiv, po.astype(np.int32))
    assert np.array_equal(F, Fo)
    b = np.random.default_rng(1).uniform(-1, 1, N)
    x = b.copy()
    I.LinearSolvers.overwriting_solve_bunch_kaufman(F, ipiv, x, ctx)
    # an indefinite system solved: residual check in fp64
    assert np.abs(K @ x - b).max() < 1e-10 * max(1.0, np.abs(K).max() * np.abs(x).max())


def test_bk_device_fix_kp(ctx):
    # device API: fix_kp=1 records kp = k for the second zero column (LAPACK),
    # info = 1 + the first zero column
    N = 16
    K = load("bkz16_K.bin").reshape(N, N)
    A = torch.from_numpy(K.copy()).cuda()
    piv = torch.zeros(N, dtype=torch.int32, device="cuda")
    info = ctx.bk_factor(N, A.data_ptr(), N, piv.data_ptr(), fix_kp=True)
    _, po, info_o = oracle.bk_factor(K, fix_kp=True)
    assert info == info_o + 1
    assert np.array_equal(piv.cpu().numpy(), po.astype(np.int32))


def test_bk_zero_column0_device_info(ctx):
    # info = 1 + the first zero column (column 0 here), while ipiv follows the
    # reference's 0-based bookkeeping bit for bit
    N = 16
    K = load("bkz0_16_K.bin").reshape(N, N)
    A = torch.from_numpy(K.copy()).cuda()
    piv = torch.zeros(N, dtype=torch.int32, device="cuda")
    info = ctx.bk_factor(N, A.data_ptr(), N, piv.data_ptr(), fix_kp=False)
    assert info == 1
    assert np.array_equal(piv.cpu().numpy(), load("bkz0_16_ipiv.bin").astype(np.int32))
    assert np.array_equal(A.cpu().numpy(), load("bkz0_16_F.bin").reshape(N, N))


# ---------------------------------------------------------------------------
# The whole-device factor (k_bk_grid: every CU, one grid barrier per pivot
# step, fixed row ownership): the same bitwise contract at any N.
def _dev_factor(ctx, K, algo, fix_kp=False):
    N = K.shape[0]
    A = torch.from_numpy(np.ascontiguousarray(K)).cuda()
    piv = torch.zeros(max(N, 1), dtype=torch.int32, device="cuda")
    info = ctx.bk_factor(N, A.data_ptr(), N, piv.data_ptr(), fix_kp=fix_kp, algo=algo)
    return A.cpu().numpy(), piv.cpu().numpy()[:N], info


@pytest.mark.parametrize("N,tag", [(8, "bk8"), (64, "bk64"), (8, "bkr8"), (64, "bkr64"), (200, "bkr200"),
                                   (16, "bkz16"), (16, "bkz0_16")])
def test_bk_grid_golden(ctx, N, tag):
    K = load(f"{tag}_K.bin").reshape(N, N)
    F, piv, info = _dev_factor(ctx, K, ctx.BK_GRID)
    assert np.array_equal(piv, load(f"{tag}_ipiv.bin").astype(np.int32))
    assert np.array_equal(F, load(f"{tag}_F.bin").reshape(N, N))  # upper triangle untouched too


def _kkt_zero_block(n, m, seed):
    # [[H, B^T], [B, 0]]: the zero block forces interchanges and 2x2 pivots
    rng = np.random.default_rng(seed)
    H = rng.uniform(-1, 1, (n, n))
    H = H + H.T
    H[np.arange(n), np.arange(n)] *= 0.01  # weak diagonal: interchanges and 2x2 pivots
    B = rng.uniform(-1, 1, (m, n))
    K = np.zeros((n + m, n + m))
    K[:n, :n] = H
    K[n:, :n] = B
    K[:n, n:] = B.T
    return K


@pytest.mark.parametrize("N,zeros", [(1, 0), (2, 0), (5, 0), (300, 0), (1000, 2), (2500, 0), (6000, 3)])
def test_bk_grid_vs_oracle_bitwise(ctx, N, zeros):
    K = _indef(N, N + 7, zeros)
    F, piv, info = _dev_factor(ctx, K, ctx.BK_GRID)
    Fo, po, io = oracle.bk_factor(K)
    assert np.array_equal(piv, po.astype(np.int32))
    assert np.array_equal(np.tril(F), np.tril(Fo))
    assert np.array_equal(np.triu(F, 1), np.triu(K, 1))
    assert info == (io + 1 if zeros else 0)


@pytest.mark.parametrize("n,m", [(700, 300), (4000, 800)])
def test_bk_grid_kkt_vs_oracle_bitwise(ctx, n, m):
    K = _kkt_zero_block(n, m, n)
    F, piv, _ = _dev_factor(ctx, K, ctx.BK_GRID)
    Fo, po, _ = oracle.bk_factor(K)
    assert (po < 0).any() and (po != np.arange(n + m)).any()  # 2x2 pivots and interchanges happened
    assert np.array_equal(piv, po.astype(np.int32))
    assert np.array_equal(np.tril(F), np.tril(Fo))


def test_bk_grid_equals_workgroup(ctx):
    K = _kkt_zero_block(1200, 400, 3)
    Fg, pg, _ = _dev_factor(ctx, K, ctx.BK_GRID)
    Fw, pw, _ = _dev_factor(ctx, K, ctx.BK_WORKGROUP)
    assert np.array_equal(pg, pw) and np.array_equal(Fg, Fw)


def test_bk_grid_fix_kp(ctx):
    N = 16
    K = load("bkz16_K.bin").reshape(N, N)
    for fix in (False, True):
        _, piv, info = _dev_factor(ctx, K, ctx.BK_GRID, fix_kp=fix)
        _, po, info_o = oracle.bk_factor(K, fix_kp=fix)
        assert info == info_o + 1
        assert np.array_equal(piv, po.astype(np.int32))


# ---------------------------------------------------------------------------
# The device-wide solve (bk_fast_*, from N = 512): the interleaved
# interchanges folded into L' once per factor, the two sweeps on the
# persistent triangular solve, D's 1x1 / 2x2 blocks in the reference's
# arithmetic (LinearSolvers.cpp:209-318).  Tolerance as the golden solves:
# 1e-12 relative to the oracle's reference-order solve.
@pytest.mark.parametrize("n,m", [(700, 300), (3000, 600)])
def test_bk_fast_solve_kkt_vs_oracle(ctx, n, m):
    K = _kkt_zero_block(n, m, n + 1)
    F, ipiv = I.LinearSolvers.symmetric_indefinite_factorization(K, ctx)
    Fo, po, _ = oracle.bk_factor(K)
    assert (po < 0).any() and (po != np.arange(n + m)).any()  # 2x2 pivots and interchanges
    assert np.array_equal(ipiv, po.astype(np.int32)) and np.array_equal(F, Fo)
    b = np.random.default_rng(2).uniform(-1, 1, n + m)
    ref = oracle.bk_solve(Fo, po, b)
    x = b.copy()
    I.LinearSolvers.overwriting_solve_bunch_kaufman(F, ipiv, x, ctx)
    assert np.abs(x - ref).max() <= 1e-12 * max(1.0, np.abs(ref).max())
    assert np.abs(K @ x - b).max() < 1e-10 * max(1.0, np.abs(K).max() * np.abs(x).max())


def test_bk_fast_solve_singular_falls_back(ctx):
    # all-zero columns: the reference divides by zero (and its kp = 0 defect
    # swaps backwards); the device solve then runs the reference's own
    # interleaved sweeps, so the non-finite entries are the oracle's
    N = 900
    K = _indef(N, 11, zeros=2)
    F, ipiv = I.LinearSolvers.symmetric_indefinite_factorization(K, ctx)
    Fo, po, _ = oracle.bk_factor(K)
    assert np.array_equal(ipiv, po.astype(np.int32))
    b = np.random.default_rng(3).uniform(-1, 1, N)
    ref = oracle.bk_solve(Fo, po, b)
    x = b.copy()
    I.LinearSolvers.overwriting_solve_bunch_kaufman(F, ipiv, x, ctx)
    assert np.array_equal(np.isfinite(x), np.isfinite(ref))
    fin = np.isfinite(ref)
    assert np.abs(x[fin] - ref[fin]).max() <= 1e-12 * max(1.0, np.abs(ref[fin]).max())
