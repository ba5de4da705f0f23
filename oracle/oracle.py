"""ctypes wrapper of the CPU oracle (oracle/libipmz_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker or the timed CPU baseline.  The
product package (ipm-zoo_amd/ipmz_amd) never imports it.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libipmz_oracle.so")

_P = ctypes.POINTER(ctypes.c_double)
_i64 = ctypes.c_int64
_u64 = ctypes.c_uint64

# Canonical slots (ipmz_oracle.cpp enum Slot / include/ipmz.h IPMZ_SLOT_*)
SLOTS = ["x", "lambda_A", "lambda_C", "s", "p", "lambda_g", "lambda_h", "lambda_y", "lambda_z",
         "g", "h", "y", "z"]
NONNEG = {"lambda_g", "lambda_h", "lambda_y", "lambda_z", "g", "h", "y", "z"}


# Settings (SymbolicOptimization.h:28-64): Bounds as bit masks 1 = Lower, 2 = Upper
# (the C ABI encodes them as IPMZ_BOUNDS_*, Both = 0; tests map between the two)
BOUNDS = {"None": 0, "Lower": 1, "Upper": 2, "Both": 3}


class Form:
    """Formulation: inequality handling (slacks=True: InequalityHandling::Slacks;
    naive=True: InequalityHandling::NaiveSlacks) and the bounds of the
    inequalities / variables (BOUNDS values)."""

    def __init__(self, slacks=False, ineq_bounds=3, var_bounds=3, naive=False):
        self.slacks = bool(slacks)
        self.naive = bool(naive)
        self.ineq_bounds = ineq_bounds
        self.var_bounds = var_bounds

    @property
    def handling(self):  # ipmzo_set_formulation / the C ABI's IPMZ_INEQ_*
        return 2 if self.naive else 1 if self.slacks else 0


def slot_size(name, n, m, p, eq_none=False, form=None):
    """eq_none: any equality handling without the slack p (None, PenaltyFunction)."""
    f = form or Form()
    vlo, vup = bool(f.var_bounds & 1), bool(f.var_bounds & 2)
    alo, aup = bool(f.ineq_bounds & 1), bool(f.ineq_bounds & 2)
    sizes = {"x": n, "lambda_y": n if vlo else 0, "lambda_z": n if vup else 0,
             "y": n if vlo and not f.slacks else 0, "z": n if vup and not f.slacks else 0,
             "lambda_A": 0 if f.naive else m, "s": 0 if f.naive else m,
             "lambda_g": m if alo else 0, "lambda_h": m if aup else 0,
             "g": m if alo and not f.slacks else 0, "h": m if aup and not f.slacks else 0}
    if name in sizes:
        return sizes[name]
    if name == "p" and eq_none:
        return 0
    return p


NAIVE_ORDER = ["x", "lambda_g", "lambda_h", "lambda_C", "p", "lambda_y", "lambda_z", "g", "h", "y", "z"]


def newton_order(n, m, p, eq_none=False, form=None):
    """Reference Newton-variable order with absent blocks dropped (NaiveSlacks:
    formulations.txt, its duals lambda_g, lambda_h ahead of lambda_C)."""
    slots = NAIVE_ORDER if form is not None and form.naive else SLOTS
    return [s for s in slots if slot_size(s, n, m, p, eq_none, form) > 0]


def _dp(a):
    return a.ctypes.data_as(_P)


def _load():
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"oracle library missing: {LIB_PATH} (run __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH)
    lib.ipmzo_create.restype = ctypes.c_void_p
    lib.ipmzo_create.argtypes = [_i64, _i64, _i64] + [_P] * 9
    lib.ipmzo_destroy.argtypes = [ctypes.c_void_p]
    lib.ipmzo_set_equality_none.argtypes = [ctypes.c_void_p]
    lib.ipmzo_set_equality_penalty.argtypes = [ctypes.c_void_p]
    lib.ipmzo_set_formulation.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.ipmzo_set_formulation.restype = ctypes.c_int
    lib.ipmzo_iterate.argtypes = [ctypes.c_void_p, _P]
    lib.ipmzo_iterate.restype = ctypes.c_int
    lib.ipmzo_iterate_timed.argtypes = [ctypes.c_void_p, _P, _P]
    lib.ipmzo_iterate_timed.restype = ctypes.c_int
    for fn in ("ipmzo_state_len", "ipmzo_kkt_dim"):
        getattr(lib, fn).restype = _i64
        getattr(lib, fn).argtypes = [ctypes.c_void_p]
    for fn in ("ipmzo_get_vars", "ipmzo_get_daff", "ipmzo_get_dir", "ipmzo_set_vars", "ipmzo_assemble"):
        getattr(lib, fn).argtypes = [ctypes.c_void_p, _P]
    lib.ipmzo_rhs.argtypes = [ctypes.c_void_p, ctypes.c_double, _P]
    for fn in ("ipmzo_residual_norm", "ipmzo_mu", "ipmzo_objective"):
        getattr(lib, fn).restype = ctypes.c_double
        getattr(lib, fn).argtypes = [ctypes.c_void_p]
    lib.ipmzo_gen_qp.argtypes = [_i64, _i64, _i64, _u64] + [_P] * 9
    lib.ipmzo_ldlt.argtypes = [_i64, _P, _i64, _P, _i64, _P]
    lib.ipmzo_ldlt_blocked.argtypes = [_i64, _P, _i64, _P, _i64, _P]
    lib.ipmzo_set_serial_ldlt.argtypes = [ctypes.c_int]
    lib.ipmzo_solve_ldlt.argtypes = [_i64, _P, _i64, _P, _P]
    lib.ipmzo_bk_factor.argtypes = [_i64, _P, _i64, ctypes.POINTER(ctypes.c_int64), ctypes.c_int]
    lib.ipmzo_bk_factor.restype = ctypes.c_int
    lib.ipmzo_bk_solve.argtypes = [_i64, _P, _i64, ctypes.POINTER(ctypes.c_int64), _P]
    lib.ipmzo_u01.restype = ctypes.c_double
    lib.ipmzo_u01.argtypes = [_u64, _u64, _u64, _u64]
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def gen_qp(n, m, p, seed):
    """Synthetic dense QP of SURVEY.md §8d (counter-based splitmix64)."""
    Q = np.zeros(n * n)
    c = np.zeros(n)
    A = np.zeros(max(m * n, 1))
    lA = np.zeros(max(m, 1))
    uA = np.zeros(max(m, 1))
    C = np.zeros(max(p * n, 1))
    d = np.zeros(max(p, 1))
    lx = np.zeros(n)
    ux = np.zeros(n)
    lib().ipmzo_gen_qp(n, m, p, seed, _dp(Q), _dp(c), _dp(A), _dp(lA), _dp(uA), _dp(C), _dp(d), _dp(lx), _dp(ux))
    return dict(n=n, m=m, p=p, Q=Q.reshape(n, n), c=c, A=A[: m * n].reshape(m, n), lA=lA[:m], uA=uA[:m],
                C=C[: p * n].reshape(p, n), d=d[:p], lx=lx, ux=ux)


def ldlt(K):
    """Restatement of LinearSolvers::ldlt_decomposition (full L, D)."""
    K = np.ascontiguousarray(K, dtype=np.float64)
    N = K.shape[0]
    L = np.zeros((N, N))
    D = np.zeros(N)
    lib().ipmzo_ldlt(N, _dp(K), N, _dp(L), N, _dp(D))
    return L, D


def ldlt_blocked(K):
    """The blocked, OpenMP-threaded form of the same factorization (bitwise
    equal to ldlt(); what OracleQP uses unless set_serial_ldlt(True))."""
    K = np.ascontiguousarray(K, dtype=np.float64)
    N = K.shape[0]
    L = np.zeros((N, N))
    D = np.zeros(N)
    lib().ipmzo_ldlt_blocked(N, _dp(K), N, _dp(L), N, _dp(D))
    return L, D


def set_serial_ldlt(serial):
    """True: OracleQP factors with the reference's own loop order on one core
    (bench.py's cpu_baseline); False (default): the blocked threaded form."""
    lib().ipmzo_set_serial_ldlt(int(bool(serial)))


def solve_ldlt(L, D, b):
    """Restatement of LinearSolvers::overwriting_solve_ldlt (returns x)."""
    L = np.ascontiguousarray(L, dtype=np.float64)
    x = np.array(b, dtype=np.float64, copy=True)
    lib().ipmzo_solve_ldlt(len(x), _dp(L), L.shape[1], _dp(np.ascontiguousarray(D, dtype=np.float64)), _dp(x))
    return x


def bk_factor(K, fix_kp=False):
    """Restatement of LinearSolvers::symmetric_indefinite_factorization
    (LinearSolvers.cpp:76-207): returns (F, ipiv, info); fix_kp=True records
    kp = k for a second zero column instead of the reference's kp = 0."""
    F = np.array(K, dtype=np.float64, copy=True, order="C")
    N = F.shape[0]
    ipiv = np.zeros(N, dtype=np.int64)
    info = lib().ipmzo_bk_factor(N, _dp(F), N, ipiv.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), int(fix_kp))
    return F, ipiv, info


def bk_solve(F, ipiv, b):
    """Restatement of LinearSolvers::overwriting_solve_bunch_kaufman
    (LinearSolvers.cpp:209-318): returns x."""
    F = np.ascontiguousarray(F, dtype=np.float64)
    ipiv = np.ascontiguousarray(ipiv, dtype=np.int64)
    x = np.array(b, dtype=np.float64, copy=True)
    lib().ipmzo_bk_solve(len(x), _dp(F), F.shape[1], ipiv.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), _dp(x))
    return x


class OracleQP:
    """CPU restatement of Optimizer (SlackedSlacks inequalities, Regularization
    equalities -- or, eq_none=True, EqualityHandling::None with the
    Bunch-Kaufman factor) from build_environment's initial iterate."""

    def __init__(self, qp, eq_none=False, eq_penalty=False, form=None):
        self.qp = qp
        self.eq_none = bool(eq_none) or bool(eq_penalty)  # no p block
        self.form = form or Form()
        n, m, p = qp["n"], qp["m"], qp["p"]
        self._keep = [np.ascontiguousarray(qp[k], dtype=np.float64).reshape(-1) if np.size(qp[k]) else np.zeros(1)
                      for k in ("Q", "c", "A", "lA", "uA", "C", "d", "lx", "ux")]
        self.h = ctypes.c_void_p(lib().ipmzo_create(n, m, p, *[_dp(a) for a in self._keep]))
        if eq_penalty:
            lib().ipmzo_set_equality_penalty(self.h)
        elif eq_none:
            lib().ipmzo_set_equality_none(self.h)
        if form is not None:
            ib = form.ineq_bounds if m else 3
            if lib().ipmzo_set_formulation(self.h, form.handling, ib, form.var_bounds) != 0:
                raise ValueError("unsupported formulation")
        self.N = lib().ipmzo_kkt_dim(self.h)
        self.L = lib().ipmzo_state_len(self.h)
        self.order = newton_order(n, m, p, self.eq_none, self.form)

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.ipmzo_destroy(self.h)

    def iterate(self):
        rec = np.zeros(8)
        conv = lib().ipmzo_iterate(self.h, _dp(rec))
        keys = ("f", "res", "mu", "alpha_aff", "mu_aff", "sigma", "alpha", "converged")
        return conv, dict(zip(keys, rec))

    def iterate_timed(self):
        """One iteration; returns (converged, record, {assemble, ldlt, rest} seconds)."""
        rec = np.zeros(8)
        ph = np.zeros(3)
        conv = lib().ipmzo_iterate_timed(self.h, _dp(rec), _dp(ph))
        return conv, rec, dict(assemble=ph[0], ldlt=ph[1], rest=ph[2])

    def _get(self, fn):
        out = np.zeros(self.L)
        getattr(lib(), fn)(self.h, _dp(out))
        return out

    def vars(self):
        return self._get("ipmzo_get_vars")

    def daff(self):
        return self._get("ipmzo_get_daff")

    def dir(self):
        return self._get("ipmzo_get_dir")

    def set_vars(self, v):
        v = np.ascontiguousarray(v, dtype=np.float64)
        lib().ipmzo_set_vars(self.h, _dp(v))

    def kkt(self):
        K = np.zeros(self.N * self.N)
        lib().ipmzo_assemble(self.h, _dp(K))
        return K.reshape(self.N, self.N)

    def rhs(self, mu=0.0):
        b = np.zeros(self.N)
        lib().ipmzo_rhs(self.h, mu, _dp(b))
        return b

    def residual_norm(self):
        return lib().ipmzo_residual_norm(self.h)

    def mu(self):
        return lib().ipmzo_mu(self.h)

    def objective(self):
        return lib().ipmzo_objective(self.h)

    def split(self, flat):
        """Split a concatenated state vector into {slot: array}."""
        n, m, p = self.qp["n"], self.qp["m"], self.qp["p"]
        out, off = {}, 0
        for s in self.order:
            k = slot_size(s, n, m, p, self.eq_none, self.form)
            out[s] = flat[off:off + k]
            off += k
        return out


def eqss_merge(qp):
    """EqualityHandling::SlackedSlacks restated as inequality rows: C x - t = 0,
    d <= t <= d, i.e. A' = [A; C], l' = [l_A; d], u' = [u_A; d], p' = 0
    (SymbolicOptimization.cpp:150-161 against 108-125; the two blocks' formulas
    are the same with l_A = u_A = d, tests/test_oracle_formulations.py)."""
    n, m, p = qp["n"], qp["m"], qp["p"]
    return dict(qp, m=m + p, p=0, A=np.vstack([qp["A"], qp["C"]]), lA=np.concatenate([qp["lA"], qp["d"]]),
                uA=np.concatenate([qp["uA"], qp["d"]]), C=np.zeros((0, n)), d=np.zeros(0))


class EqSlackedOracle:
    """OracleQP over eqss_merge(qp), in the reference's variable order
    (x, lambda_A, lambda_C, s, t, lambda_g, lambda_h, lambda_v, lambda_w,
    lambda_y, lambda_z, g, h, v, w, y, z) and with t starting at 1
    (EnvironmentBuilder.cpp:62), as capi.cpp's eqss_perm.

    naive=True: EqualityHandling::NaiveSlacks with NaiveSlacks inequalities
    (SymbolicOptimization.cpp:163-171 against 104-116: C x - v = d, C x + w = d
    are the inequality rows A x - g = l, A x + h = u with l = u = d), order x,
    lambda_g, lambda_h, lambda_v, lambda_w, lambda_y, lambda_z, g, h, v, w, y, z
    (v, w and their duals start at 1 like g, h)."""

    def __init__(self, qp, naive=False):
        n, m, p = qp["n"], qp["m"], qp["p"]
        self.qp = qp
        self.o = OracleQP(eqss_merge(qp), form=Form(naive=True) if naive else None)
        mp = m + p
        off = n if naive else n + 2 * mp
        perm = list(range(off))  # x (, [lambda_A lambda_C], [s t])
        for base in (off, off + 2 * mp + 2 * n):  # [lambda_g lambda_v][lambda_h lambda_w], then [g v][h w]
            perm += list(range(base, base + m)) + list(range(base + mp, base + mp + m))
            perm += list(range(base + m, base + mp)) + list(range(base + mp + m, base + 2 * mp))
            if base == off:
                perm += list(range(off + 2 * mp, off + 2 * mp + 2 * n))  # lambda_y, lambda_z
        perm += list(range(len(perm), self.o.L))  # y, z
        self.perm = np.array(perm)
        assert sorted(perm) == list(range(self.o.L))
        # KKT rows: x, [lambda_A lambda_C] already in the reference's order;
        # NaiveSlacks: x, [lambda_g lambda_v], [lambda_h lambda_w] -> x,
        # lambda_g, lambda_h, lambda_v, lambda_w
        self.kperm = np.array(perm[:self.o.N]) if naive else np.arange(self.o.N)
        self.N, self.L = self.o.N, self.o.L
        self.sizes = dict(x=n, lambda_A=0 if naive else m, lambda_C=0 if naive else p, s=0 if naive else m,
                          t=0 if naive else p, lambda_g=m, lambda_h=m, lambda_v=p, lambda_w=p,
                          lambda_y=n, lambda_z=n, g=m, h=m, v=p, w=p, y=n, z=n)
        self.order = [k for k in self.sizes if self.sizes[k]]
        if not naive:
            v = self.o.vars()
            v[n + 2 * m + p: n + 2 * mp] = 1.0  # t
            self.o.set_vars(v)

    def vars(self):
        return self.o.vars()[self.perm]

    def daff(self):
        return self.o.daff()[self.perm]

    def dir(self):
        return self.o.dir()[self.perm]

    def set_vars(self, v):
        w = np.empty(self.L)
        w[self.perm] = v
        self.o.set_vars(w)

    def iterate(self):
        return self.o.iterate()

    def kkt(self):
        K = self.o.kkt()
        return K[np.ix_(self.kperm, self.kperm)]

    def split(self, flat):
        out, off = {}, 0
        for s in self.order:
            out[s] = flat[off:off + self.sizes[s]]
            off += self.sizes[s]
        return out
