"""Python binding of libipmz (the MI355X Newton-step library) over its C ABI
(include/ipmz.h), via ctypes.

Mirrors the reference's NumericalOptimization interface for the hot path:

    LinearSolvers.ldlt_decomposition(A)        -> (L, D)   LinearSolvers.h:11
    LinearSolvers.overwriting_solve_ldlt(L, D, b)  (b overwritten)  LinearSolvers.h:16-17
    Data / build_environment / Optimizer(...).solve()     EnvironmentBuilder.h:7-20,
                                                           Optimizer.h:15-20

Errors raise AssertionError (a subclass of the reference's
Utils::AssertionError -> std::logic_error convention, Assert.h:7-12, maps to
Python's AssertionError/ValueError family here).  There is no CPU fallback:
loading fails loudly when lib/libipmz.so is missing, and every computing
call fails when no gfx950 device is visible.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(HERE), "lib", "libipmz.so")

IPMZ_OK = 0
ERR = {-1: "invalid argument", -2: "HIP error", -3: "out of device memory", -4: "no gfx950 device",
       -5: "bad state"}
SC = dict(f=0, res=1, mu=2, alpha_aff=3, mu_aff=4, sigma=5, alpha=6, converged=7, mu_new=8, restarts=9,
          ir_ratio_aff=10, ir_iters_aff=11, ir_ratio=12, ir_iters=13)
SC_COUNT = 16
PH = dict(step=0, assemble=1, factor=2, solve=3, trailing=4, eval=5)
STEP_RESTART_IF_CONVERGED = 1
STEP_GRAPH = 2
SLOTS = ["x", "lambda_A", "lambda_C", "s", "p", "lambda_g", "lambda_h", "lambda_y", "lambda_z", "g", "h", "y", "z"]

EXPORTS = [
    "ipmz_ctx_create", "ipmz_ctx_destroy", "ipmz_ctx_set_stream", "ipmz_ctx_reset_stream", "ipmz_ctx_sync", "ipmz_last_error",
    "ipmz_ctx_set_blocking", "ipmz_ctx_get_blocking", "ipmz_ldlt_workspace_bytes", "ipmz_ldlt_factor", "ipmz_ldlt_solve",
    "ipmz_ldlt_prepare_solve", "ipmz_ldlt_decomposition", "ipmz_overwriting_solve_ldlt", "ipmz_qp_create",
    "ipmz_qp_destroy", "ipmz_qp_load_host", "ipmz_qp_generate", "ipmz_qp_step", "ipmz_qp_scalars",
    "ipmz_qp_device_scalars", "ipmz_qp_copy_scalars", "ipmz_qp_solve", "ipmz_qp_state_len", "ipmz_qp_get_state", "ipmz_qp_set_state",
    "ipmz_qp_get_kkt", "ipmz_qp_kkt_dim", "ipmz_qp_set_timing", "ipmz_qp_phase_times",
    "ipmz_batch_create", "ipmz_batch_size", "ipmz_batch_load_host", "ipmz_batch_initialize", "ipmz_batch_scalars",
    "ipmz_batch_get_state", "ipmz_batch_set_state", "ipmz_batch_solve",
    "ipmz_mixed_workspace_bytes", "ipmz_mixed_factor", "ipmz_mixed_solve", "ipmz_qp_set_mixed_precision",
    "ipmz_batch_copy_scalars", "ipmz_normal_workspace_bytes", "ipmz_normal_factor", "ipmz_normal_solve",
    "ipmz_qp_set_reduction", "ipmz_bk_factor", "ipmz_bk_factor_ex", "ipmz_bk_solve", "ipmz_symmetric_indefinite_factorization",
    "ipmz_overwriting_solve_bunch_kaufman", "ipmz_debug_inject", "ipmz_batch_summary", "ipmz_batch_set_factor_kernel",
    "ipmz_qp_last_step_graph",
]
REDUCTION_AUGMENTED, REDUCTION_NORMAL = 0, 1

_P = ctypes.POINTER(ctypes.c_double)
_VP = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64


class IpmzError(AssertionError):
    """A failed libipmz call (the reference throws Utils::AssertionError)."""


EQ_REGULARIZATION = 0  # Settings::EqualityHandling::Regularization (include/ipmz.h IPMZ_EQ_*)
EQ_NONE = 1            # zero (lambda_C, lambda_C) block, Bunch-Kaufman factor
EQ_PENALTY = 2         # PenaltyFunction: -mu (lambda_C, lambda_C) block, LDL^T
EQ_PENALTY_EXTRA_DUAL = 3  # PenaltyFunctionWithExtraDual: the same Newton system (reference-derived)
EQ_SLACKED_SLACKS = 4  # t, v = t - d, w = d - t with duals lambda_v, lambda_w (SlackedSlacks inequalities)
EQ_NAIVE_SLACKS = 5    # C x - v = d, C x + w = d, lambda_v / lambda_w as KKT rows (NaiveSlacks inequalities)
INEQ_SLACKED_SLACKS = 0  # Settings::InequalityHandling (include/ipmz.h IPMZ_INEQ_*)
INEQ_SLACKS = 1          # no g/h/y/z slacks (the reference's corrector defect reproduced)
INEQ_NAIVE_SLACKS = 2    # no s; lambda_g, lambda_h as KKT rows (N = n + 2m + p)
BOUNDS_BOTH = 0          # Settings::Bounds (include/ipmz.h IPMZ_BOUNDS_*)
BOUNDS_LOWER = 1
BOUNDS_UPPER = 2
BOUNDS_NONE = 3


class _QPConfig(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("m", ctypes.c_int), ("p", ctypes.c_int), ("delta", ctypes.c_double),
                ("equality_handling", ctypes.c_int), ("inequality_handling", ctypes.c_int),
                ("inequality_bounds", ctypes.c_int), ("variable_bounds", ctypes.c_int)]


def _load():
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64, and
    # a second copy loaded next to it cannot open the device.  Loading torch
    # first makes libipmz bind to torch's copy (same soname), so device
    # pointers and streams are shared.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libipmz not built: {LIB_PATH} missing (run __graft_entry__.build()); "
                          "there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    sig = {
        "ipmz_ctx_create": ([ctypes.POINTER(_VP), _I], _I),
        "ipmz_ctx_destroy": ([_VP], _I),
        "ipmz_ctx_set_stream": ([_VP, _VP], _I),
        "ipmz_ctx_reset_stream": ([_VP], _I),
        "ipmz_ctx_sync": ([_VP], _I),
        "ipmz_last_error": ([], ctypes.c_char_p),
        "ipmz_ctx_set_blocking": ([_VP, _I, _I], _I),
        "ipmz_ctx_get_blocking": ([_VP, _I, ctypes.POINTER(_I), ctypes.POINTER(_I)], _I),
        "ipmz_ldlt_workspace_bytes": ([_VP, _I], _I64),
        "ipmz_ldlt_factor": ([_VP, _I, _VP, _I64, _VP, _VP, _I64], _I),
        "ipmz_ldlt_solve": ([_VP, _I, _VP, _I64, _VP, _VP, _VP], _I),
        "ipmz_ldlt_prepare_solve": ([_VP, _I, _VP, _I64, _VP, _I64], _I),
        "ipmz_ldlt_decomposition": ([_VP, _I, _P, _P, _P], _I),
        "ipmz_overwriting_solve_ldlt": ([_VP, _I, _P, _P, _P], _I),
        "ipmz_qp_create": ([_VP, ctypes.POINTER(_QPConfig), ctypes.POINTER(_VP)], _I),
        "ipmz_qp_destroy": ([_VP], _I),
        "ipmz_qp_load_host": ([_VP] + [_P] * 9, _I),
        "ipmz_qp_generate": ([_VP, ctypes.c_uint64], _I),
        "ipmz_qp_step": ([_VP, _I], _I),
        "ipmz_qp_scalars": ([_VP, _P], _I),
        "ipmz_qp_device_scalars": ([_VP, ctypes.POINTER(_VP)], _I),
        "ipmz_qp_copy_scalars": ([_VP, _VP], _I),
        "ipmz_qp_solve": ([_VP, _I, _P, ctypes.POINTER(_I)], _I),
        "ipmz_qp_state_len": ([_VP], _I64),
        "ipmz_qp_get_state": ([_VP, _I, _P], _I),
        "ipmz_qp_set_state": ([_VP, _P], _I),
        "ipmz_qp_get_kkt": ([_VP, _P], _I),
        "ipmz_qp_kkt_dim": ([_VP], _I),
        "ipmz_qp_set_timing": ([_VP, _I], _I),
        "ipmz_qp_phase_times": ([_VP, _P, _P, ctypes.POINTER(_I64)], _I),
        "ipmz_batch_create": ([_VP, ctypes.POINTER(_QPConfig), _I, ctypes.POINTER(_VP)], _I),
        "ipmz_batch_size": ([_VP], _I),
        "ipmz_batch_load_host": ([_VP, _I] + [_P] * 9, _I),
        "ipmz_batch_initialize": ([_VP], _I),
        "ipmz_batch_scalars": ([_VP, _P], _I),
        "ipmz_batch_get_state": ([_VP, _I, _I, _P], _I),
        "ipmz_batch_set_state": ([_VP, _I, _P], _I),
        "ipmz_batch_solve": ([_VP, _I, ctypes.POINTER(_I), ctypes.POINTER(_I)], _I),
        "ipmz_mixed_workspace_bytes": ([_VP, _I], _I64),
        "ipmz_mixed_factor": ([_VP, _I, _VP, _I64, _VP, _I64], _I),
        "ipmz_mixed_solve": ([_VP, _I, _VP, _I64, _VP, _VP, ctypes.c_double, _I, _P], _I),
        "ipmz_qp_set_mixed_precision": ([_VP, _I, ctypes.c_double, _I], _I),
        "ipmz_batch_copy_scalars": ([_VP, _VP], _I),
        "ipmz_normal_workspace_bytes": ([_VP, _I, _I], _I64),
        "ipmz_normal_factor": ([_VP, _I, _I, _VP, _I64, _VP, _VP, _I64], _I),
        "ipmz_normal_solve": ([_VP, _I, _I, _VP, _I64, _VP, _VP, _VP], _I),
        "ipmz_qp_set_reduction": ([_VP, _I], _I),
        "ipmz_bk_factor": ([_VP, _I, _VP, _I64, _VP, _I], _I),
        "ipmz_bk_factor_ex": ([_VP, _I, _VP, _I64, _VP, _I, _I], _I),
        "ipmz_bk_solve": ([_VP, _I, _VP, _I64, _VP, _VP], _I),
        "ipmz_symmetric_indefinite_factorization": ([_VP, _I, _P, _P, ctypes.POINTER(ctypes.c_int)], _I),
        "ipmz_overwriting_solve_bunch_kaufman": ([_VP, _I, _P, ctypes.POINTER(ctypes.c_int), _P], _I),
        "ipmz_debug_inject": ([_I], _I),
        "ipmz_batch_summary": ([_VP, _VP], _I),
        "ipmz_batch_set_factor_kernel": ([_VP, _I], _I),
        "ipmz_qp_last_step_graph": ([_VP], _I),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    return lib


lib = _load()


def _check(rc, what):
    if rc < 0:
        msg = lib.ipmz_last_error().decode(errors="replace")
        raise IpmzError(f"{what}: {ERR.get(rc, rc)}: {msg}")
    return rc


def _dp(a):
    return a.ctypes.data_as(_P)


class Context:
    """A device + HIP stream (one per GPU / process)."""

    def __init__(self, device=0, stream=None, nbo=None, nbi=None):
        h = _VP()
        _check(lib.ipmz_ctx_create(ctypes.byref(h), device), "ipmz_ctx_create")
        self.h = h
        self.device = device
        self.stream = None  # None: the context's own (non-blocking) stream
        if stream is not None:
            self.set_stream(stream)
        if nbo or nbi:  # nbo 0 / None: by matrix order (libipmz's default)
            self.set_blocking(nbo or 0, nbi or 64)

    def set_stream(self, stream):
        """Enqueue on an external HIP stream handle (0 = the null stream,
        which is PyTorch's default stream); None = the context's own stream."""
        if stream is None:
            _check(lib.ipmz_ctx_reset_stream(self.h), "ipmz_ctx_reset_stream")
        else:
            _check(lib.ipmz_ctx_set_stream(self.h, _VP(stream)), "ipmz_ctx_set_stream")
        self.stream = stream

    def on_stream(self, stream):
        """True when work enqueued on this context is ordered before later
        work on the HIP stream handle `stream` (the same stream)."""
        return self.stream is not None and int(self.stream) == int(stream)

    def set_blocking(self, nbo, nbi):
        _check(lib.ipmz_ctx_set_blocking(self.h, nbo, nbi), "ipmz_ctx_set_blocking")

    def blocking(self, N):
        """(nbo, nbi) an order-N factor uses with this context."""
        nbo, nbi = _I(0), _I(0)
        _check(lib.ipmz_ctx_get_blocking(self.h, N, ctypes.byref(nbo), ctypes.byref(nbi)), "ipmz_ctx_get_blocking")
        return nbo.value, nbi.value

    def sync(self):
        """Synchronize; raises IpmzError when the last device-memory factor /
        solve hit a hand-off timeout (its sticky error words)."""
        _check(lib.ipmz_ctx_sync(self.h), "ipmz_ctx_sync")

    def close(self):
        if getattr(self, "h", None):
            lib.ipmz_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- device-memory LinearSolvers (pointers, e.g. torch tensor data_ptr()) --
    def workspace_bytes(self, N):
        return lib.ipmz_ldlt_workspace_bytes(self.h, N)

    def ldlt_factor(self, N, K_ptr, ld, D_ptr, ws_ptr, ws_bytes):
        return _check(lib.ipmz_ldlt_factor(self.h, N, _VP(K_ptr), ld, _VP(D_ptr), _VP(ws_ptr), ws_bytes),
                      "ipmz_ldlt_factor")

    def ldlt_solve(self, N, K_ptr, ld, D_ptr, ws_ptr, b_ptr):
        return _check(lib.ipmz_ldlt_solve(self.h, N, _VP(K_ptr), ld, _VP(D_ptr), _VP(ws_ptr), _VP(b_ptr)),
                      "ipmz_ldlt_solve")

    # -- mixed precision (C5): fp32 factor of S K S + fp64 refinement --
    def mixed_workspace_bytes(self, N):
        return lib.ipmz_mixed_workspace_bytes(self.h, N)

    def mixed_factor(self, N, K_ptr, ld, ws_ptr, ws_bytes):
        return _check(lib.ipmz_mixed_factor(self.h, N, _VP(K_ptr), ld, _VP(ws_ptr), ws_bytes), "ipmz_mixed_factor")

    def mixed_solve(self, N, K_ptr, ld, ws_ptr, b_ptr, tol=1e-12, max_refine=10):
        """b <- K^{-1} b (device pointers); returns (ratio reached, corrections)."""
        stat = np.zeros(2)
        _check(lib.ipmz_mixed_solve(self.h, N, _VP(K_ptr), ld, _VP(ws_ptr), _VP(b_ptr), tol, max_refine, _dp(stat)),
               "ipmz_mixed_solve")
        return float(stat[0]), int(stat[1])

    # -- Bunch-Kaufman on device memory (f3) --
    BK_AUTO, BK_WORKGROUP, BK_GRID = 0, 1, 2

    def bk_factor(self, N, A_ptr, ld, ipiv_ptr, fix_kp=False, algo=0):
        """symmetric_indefinite_factorization in place (LinearSolvers.cpp:76-207);
        algo: BK_AUTO, BK_WORKGROUP (one workgroup, N <= 4096) or BK_GRID (every CU)."""
        return _check(lib.ipmz_bk_factor_ex(self.h, N, _VP(A_ptr), ld, _VP(ipiv_ptr), int(fix_kp), int(algo)),
                      "ipmz_bk_factor")

    def bk_solve(self, N, F_ptr, ld, ipiv_ptr, b_ptr):
        return _check(lib.ipmz_bk_solve(self.h, N, _VP(F_ptr), ld, _VP(ipiv_ptr), _VP(b_ptr)), "ipmz_bk_solve")

    # -- normal equations (C2) --
    def normal_workspace_bytes(self, n, mp):
        return lib.ipmz_normal_workspace_bytes(self.h, n, mp)

    def normal_factor(self, n, mp, K_ptr, ld, D_ptr, ws_ptr, ws_bytes):
        return _check(lib.ipmz_normal_factor(self.h, n, mp, _VP(K_ptr), ld, _VP(D_ptr), _VP(ws_ptr), ws_bytes),
                      "ipmz_normal_factor")

    def normal_solve(self, n, mp, K_ptr, ld, D_ptr, ws_ptr, b_ptr):
        return _check(lib.ipmz_normal_solve(self.h, n, mp, _VP(K_ptr), ld, _VP(D_ptr), _VP(ws_ptr), _VP(b_ptr)),
                      "ipmz_normal_solve")


def debug_inject(mask):
    """Test hook (ipmz_debug_inject): 1 = drop the persistent solve's first
    hand-off, 2 = the outer-panel factor's; 0 = normal operation."""
    _check(lib.ipmz_debug_inject(int(mask)), "ipmz_debug_inject")


INJECT_SOLVE, INJECT_PANEL, INJECT_GRAPH_FORKS = 1, 2, 4

_default_ctx = None


def default_context():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


class LinearSolvers:
    """NumericalOptimization::LinearSolvers with the reference's value semantics
    (LinearSolvers.h:11-17): fresh L and D returned, b overwritten."""

    @staticmethod
    def ldlt_decomposition(A, ctx=None):
        A = np.ascontiguousarray(A, dtype=np.float64)
        if A.ndim != 2 or A.shape[0] != A.shape[1]:
            raise IpmzError("ldlt_decomposition: matrix must be square")  # LinearSolvers.cpp:16-17
        N = A.shape[0]
        L = np.zeros((N, N))
        D = np.zeros(N)
        info = _check(lib.ipmz_ldlt_decomposition((ctx or default_context()).h, N, _dp(A), _dp(L), _dp(D)),
                      "ipmz_ldlt_decomposition")
        return L, D, info

    @staticmethod
    def overwriting_solve_ldlt(L, D, b, ctx=None):
        L = np.ascontiguousarray(L, dtype=np.float64)
        D = np.ascontiguousarray(D, dtype=np.float64)
        if not (isinstance(b, np.ndarray) and b.dtype == np.float64 and b.flags.c_contiguous):
            raise IpmzError("overwriting_solve_ldlt: b must be a contiguous float64 array")
        N = b.shape[0]
        if N and (D.shape[0] != N or L.shape != (N, N)):
            raise IpmzError("overwriting_solve_ldlt: size mismatch")  # LinearSolvers.cpp:50-53
        _check(lib.ipmz_overwriting_solve_ldlt((ctx or default_context()).h, N, _dp(L), _dp(D), _dp(b)),
               "ipmz_overwriting_solve_ldlt")
        return b


def _ip(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


def symmetric_indefinite_factorization(A, ctx=None):
    """LinearSolvers::symmetric_indefinite_factorization (LinearSolvers.h:23-26):
    returns (F, ipiv) -- F is A with its lower triangle factored."""
    A = np.ascontiguousarray(A, dtype=np.float64)
    if A.ndim != 2 or A.shape[0] != A.shape[1]:
        raise IpmzError("symmetric_indefinite_factorization: matrix must be square")
    N = A.shape[0]
    F = np.zeros((N, N))
    ipiv = np.zeros(N, dtype=np.int32)
    _check(lib.ipmz_symmetric_indefinite_factorization((ctx or default_context()).h, N, _dp(A), _dp(F), _ip(ipiv)),
           "ipmz_symmetric_indefinite_factorization")
    return F, ipiv


def overwriting_solve_bunch_kaufman(F, ipiv, b, ctx=None):
    """LinearSolvers::overwriting_solve_bunch_kaufman (LinearSolvers.h:28-31): b overwritten."""
    F = np.ascontiguousarray(F, dtype=np.float64)
    ipiv = np.ascontiguousarray(ipiv, dtype=np.int32)
    if b.dtype != np.float64 or not b.flags.c_contiguous:
        raise IpmzError("overwriting_solve_bunch_kaufman: b must be a contiguous float64 array")
    _check(lib.ipmz_overwriting_solve_bunch_kaufman((ctx or default_context()).h, len(b), _dp(F), _ip(ipiv), _dp(b)),
           "ipmz_overwriting_solve_bunch_kaufman")


LinearSolvers.symmetric_indefinite_factorization = staticmethod(symmetric_indefinite_factorization)
LinearSolvers.overwriting_solve_bunch_kaufman = staticmethod(overwriting_solve_bunch_kaufman)


class Data:
    """NumericalOptimization::Data (EnvironmentBuilder.h:7-17)."""

    def __init__(self, Q, c, l_x, u_x, A_ineq=None, l_A_ineq=None, u_A_ineq=None, A_eq=None, b_eq=None):
        self.Q = np.ascontiguousarray(Q, dtype=np.float64)
        self.c = np.ascontiguousarray(c, dtype=np.float64)
        self.l_x = np.ascontiguousarray(l_x, dtype=np.float64)
        self.u_x = np.ascontiguousarray(u_x, dtype=np.float64)
        n = self.Q.shape[0]
        self.A_ineq = np.zeros((0, n)) if A_ineq is None else np.ascontiguousarray(A_ineq, dtype=np.float64)
        self.l_A_ineq = np.zeros(0) if l_A_ineq is None else np.ascontiguousarray(l_A_ineq, dtype=np.float64)
        self.u_A_ineq = np.zeros(0) if u_A_ineq is None else np.ascontiguousarray(u_A_ineq, dtype=np.float64)
        self.A_eq = np.zeros((0, n)) if A_eq is None else np.ascontiguousarray(A_eq, dtype=np.float64)
        self.b_eq = np.zeros(0) if b_eq is None else np.ascontiguousarray(b_eq, dtype=np.float64)


class Optimizer:
    """The Newton-step solver: build_environment + Optimizer (Optimizer.h:15-20).

    Formulation (Settings, SymbolicOptimization.h:28-64): by default
    InequalityHandling::SlackedSlacks with Bounds::Both, and
    EqualityHandling::Regularization (delta = 1e-4) when equalities exist.
    equality_handling=EQ_NONE: the zero (lambda_C, lambda_C) block the
    reference routes to solve_indefinite_ (Optimizer.cpp:63-75), factored
    with Bunch-Kaufman (any N; N <= 4096 per QP in batches); EQ_PENALTY: PenaltyFunction.
    inequality_handling=INEQ_SLACKS, inequality_bounds / variable_bounds =
    BOUNDS_LOWER / UPPER / NONE select the other Newton systems (absent
    blocks dropped from the Newton order, as the reference does).
    """

    def __init__(self, n, m=0, p=0, ctx=None, delta=1e-4, equality_handling=0, inequality_handling=0,
                 inequality_bounds=0, variable_bounds=0):
        self.ctx = ctx or default_context()
        cfg = _QPConfig(n, m, p, delta, equality_handling, inequality_handling, inequality_bounds, variable_bounds)
        self.equality_handling = equality_handling
        self.form = (inequality_handling, inequality_bounds, variable_bounds)
        h = _VP()
        _check(lib.ipmz_qp_create(self.ctx.h, ctypes.byref(cfg), ctypes.byref(h)), "ipmz_qp_create")
        self.h = h
        self.n, self.m, self.p = n, m, p
        self.N = lib.ipmz_qp_kkt_dim(h)  # n + m + p, or n + 2m + p (NaiveSlacks)
        self.state_len = lib.ipmz_qp_state_len(h)

    @classmethod
    def from_data(cls, data, ctx=None, **form):
        n, m, p = data.Q.shape[0], data.A_ineq.shape[0], data.A_eq.shape[0]
        o = cls(n, m, p, ctx, **form)
        o.load(data)
        return o

    def load(self, data):
        keep = [data.Q, data.c, data.A_ineq, data.l_A_ineq, data.u_A_ineq, data.A_eq, data.b_eq, data.l_x, data.u_x]
        keep = [np.ascontiguousarray(a, dtype=np.float64).reshape(-1) if np.size(a) else np.zeros(1) for a in keep]
        _check(lib.ipmz_qp_load_host(self.h, *[_dp(a) for a in keep]), "ipmz_qp_load_host (build_environment)")

    def generate(self, seed):
        _check(lib.ipmz_qp_generate(self.h, seed), "ipmz_qp_generate")

    def step(self, flags=0):
        _check(lib.ipmz_qp_step(self.h, flags), "ipmz_qp_step")

    def last_step_graph(self):
        """True when the last step replayed a captured hipGraph."""
        return bool(lib.ipmz_qp_last_step_graph(self.h))

    def set_reduction(self, reduction):
        """REDUCTION_AUGMENTED (default) or REDUCTION_NORMAL (config C2)."""
        _check(lib.ipmz_qp_set_reduction(self.h, reduction), "ipmz_qp_set_reduction")

    def set_mixed_precision(self, enable=True, tol=1e-12, max_refine=10):
        """Newton directions via the fp32 factor + fp64 refinement (config C5)."""
        _check(lib.ipmz_qp_set_mixed_precision(self.h, int(enable), tol, max_refine), "ipmz_qp_set_mixed_precision")

    def scalars(self):
        out = np.zeros(SC_COUNT)
        _check(lib.ipmz_qp_scalars(self.h, _dp(out)), "ipmz_qp_scalars")
        return {k: out[i] for k, i in SC.items()}

    def device_scalars_ptr(self):
        p = _VP()
        _check(lib.ipmz_qp_device_scalars(self.h, ctypes.byref(p)), "ipmz_qp_device_scalars")
        return p.value

    def copy_scalars(self, dst_ptr):
        """Async device-to-device copy of the scalar block (ctx stream)."""
        _check(lib.ipmz_qp_copy_scalars(self.h, _VP(dst_ptr)), "ipmz_qp_copy_scalars")

    def solve(self, max_iter=100):
        trace = np.zeros((max_iter + 1, 8))
        it = ctypes.c_int(0)
        _check(lib.ipmz_qp_solve(self.h, max_iter, _dp(trace), ctypes.byref(it)), "ipmz_qp_solve")
        rows = min(it.value + 1, max_iter)
        keys = ("f", "res", "mu", "alpha_aff", "mu_aff", "sigma", "alpha", "converged")
        return it.value, [dict(zip(keys, r)) for r in trace[:rows]]

    def _state(self, which):
        out = np.zeros(self.state_len)
        _check(lib.ipmz_qp_get_state(self.h, which, _dp(out)), "ipmz_qp_get_state")
        return out

    def vars(self):
        return self._state(0)

    def daff(self):
        return self._state(1)

    def dir(self):
        return self._state(2)

    def residuals(self):
        return self._state(3)

    def set_vars(self, v):
        v = np.ascontiguousarray(v, dtype=np.float64)
        _check(lib.ipmz_qp_set_state(self.h, _dp(v)), "ipmz_qp_set_state")

    def kkt(self):
        K = np.zeros((self.N, self.N))
        _check(lib.ipmz_qp_get_kkt(self.h, _dp(K)), "ipmz_qp_get_kkt")
        return K

    def set_timing(self, on=True):
        _check(lib.ipmz_qp_set_timing(self.h, 1 if on else 0), "ipmz_qp_set_timing")

    def phase_times(self):
        ms = np.zeros(8)
        fl = ctypes.c_double(0)
        nl = ctypes.c_int64(0)
        _check(lib.ipmz_qp_phase_times(self.h, _dp(ms), ctypes.byref(fl), ctypes.byref(nl)), "ipmz_qp_phase_times")
        out = {k: ms[i] for k, i in PH.items()}
        out["trailing_flops"] = fl.value
        out["trailing_launches"] = nl.value
        return out

    def close(self):
        if getattr(self, "h", None):
            lib.ipmz_qp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Batch(Optimizer):
    """A batch of independent QPs with identical (n, m, p) (config C4): every
    kernel launch serves the whole batch.  QP i of generate(seed) uses
    seed + i."""

    def __init__(self, n, m=0, p=0, batch=1, ctx=None, delta=1e-4, equality_handling=0, inequality_handling=0,
                 inequality_bounds=0, variable_bounds=0):
        self.ctx = ctx or default_context()
        cfg = _QPConfig(n, m, p, delta, equality_handling, inequality_handling, inequality_bounds, variable_bounds)
        self.equality_handling = equality_handling
        self.form = (inequality_handling, inequality_bounds, variable_bounds)
        h = _VP()
        _check(lib.ipmz_batch_create(self.ctx.h, ctypes.byref(cfg), batch, ctypes.byref(h)), "ipmz_batch_create")
        self.h = h
        self.n, self.m, self.p = n, m, p
        self.N = lib.ipmz_qp_kkt_dim(h)  # n + m + p, or n + 2m + p (NaiveSlacks)
        self.batch = batch
        self.state_len = lib.ipmz_qp_state_len(h)

    def load_one(self, index, data):
        keep = [data.Q, data.c, data.A_ineq, data.l_A_ineq, data.u_A_ineq, data.A_eq, data.b_eq, data.l_x, data.u_x]
        keep = [np.ascontiguousarray(a, dtype=np.float64).reshape(-1) if np.size(a) else np.zeros(1) for a in keep]
        _check(lib.ipmz_batch_load_host(self.h, index, *[_dp(a) for a in keep]), "ipmz_batch_load_host")

    def initialize(self):
        _check(lib.ipmz_batch_initialize(self.h), "ipmz_batch_initialize")

    def copy_batch_scalars(self, dst_ptr):
        """Async device copy of all batch x SC_COUNT scalars (ctx stream)."""
        _check(lib.ipmz_batch_copy_scalars(self.h, _VP(dst_ptr)), "ipmz_batch_copy_scalars")

    def summary(self, dst_ptr):
        """Enqueue the convergence summary {max res, max mu, unconverged}
        into 3 device doubles at dst_ptr (one kernel, ctx stream)."""
        _check(lib.ipmz_batch_summary(self.h, _VP(dst_ptr)), "ipmz_batch_summary")

    def summary_into(self, t):
        """Device tensor t (>= 3 float64): the summary (the stepper protocol
        of ipmz_amd.dist.solve_sharded).  It is ordered before anything later
        on torch's current stream: enqueued there when the context runs on
        that stream, otherwise the context's stream is synchronized after it,
        so an all-reduce or .tolist() on torch's stream never reads a stale
        buffer."""
        self.summary(t.data_ptr())
        import torch
        if not self.ctx.on_stream(torch.cuda.current_stream(t.device).cuda_stream):
            self.ctx.sync()

    FACTOR_AUTO, FACTOR_ONE, FACTOR_PAIR, FACTOR_LEFT = 0, 1, 2, 3  # include/ipmz.h IPMZ_BATCH_FACTOR_*

    def set_factor_kernel(self, kernel):
        """FACTOR_AUTO, FACTOR_ONE (right-looking, one workgroup per QP),
        FACTOR_PAIR (right-looking, two per QP; needs 2 * batch <= #CU) or
        FACTOR_LEFT (left-looking, one per QP): the small batched LDL^T kernel."""
        _check(lib.ipmz_batch_set_factor_kernel(self.h, int(kernel)), "ipmz_batch_set_factor_kernel")

    def batch_scalars(self):
        out = np.zeros(self.batch * SC_COUNT)
        _check(lib.ipmz_batch_scalars(self.h, _dp(out)), "ipmz_batch_scalars")
        return out.reshape(self.batch, SC_COUNT)

    def state(self, index, which=0):
        out = np.zeros(self.state_len)
        _check(lib.ipmz_batch_get_state(self.h, index, which, _dp(out)), "ipmz_batch_get_state")
        return out

    def set_state(self, index, v):
        v = np.ascontiguousarray(v, dtype=np.float64)
        _check(lib.ipmz_batch_set_state(self.h, index, _dp(v)), "ipmz_batch_set_state")

    def solve_all(self, max_iter=100):
        it = ctypes.c_int(0)
        nc = ctypes.c_int(0)
        _check(lib.ipmz_batch_solve(self.h, max_iter, ctypes.byref(it), ctypes.byref(nc)), "ipmz_batch_solve")
        return it.value, nc.value
