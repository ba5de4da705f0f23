/*
 * ipmz.h -- C ABI of libipmz, the MI355X (gfx950) implementation of
 * ipm-zoo's numerical interior-point Newton step.
 *
 * Drop-in boundary.  The reference has no FFI: its hot path
 * is a set of C++ free functions plus one class, all called from Optimizer.
 * Each entry point below replaces one of them:
 *
 *   ipmz_ldlt_decomposition     <- LinearSolvers::ldlt_decomposition
 *                                  (include/NumericalOptimization/LinearSolvers.h:11,
 *                                   src/NumericalOptimization/LinearSolvers.cpp:14-42)
 *   ipmz_overwriting_solve_ldlt <- LinearSolvers::overwriting_solve_ldlt
 *                                  (LinearSolvers.h:16-17, LinearSolvers.cpp:44-74)
 *   ipmz_ldlt_factor / _solve   <- the same pair on device-resident K (no copies)
 *   ipmz_qp_create + ipmz_qp_load_host
 *                               <- NumericalOptimization::build_environment
 *                                  (EnvironmentBuilder.h:19-20, EnvironmentBuilder.cpp:7-76)
 *                                  + Optimizer::Optimizer (Optimizer.h:15-18)
 *   ipmz_qp_step                <- one body of Optimizer::solve_quasi_definite_
 *                                  (Optimizer.cpp:127-219): assembly
 *                                  (get_as_matrix_, :387-391), factor, two
 *                                  compute_search_direction_ (:344-380), two
 *                                  get_max_step_ (:270-342), update (:222-231)
 *   ipmz_qp_solve               <- Optimizer::solve (Optimizer.h:20, Optimizer.cpp:63-73)
 *
 * Conventions
 *   - Plain pointers and sizes only.  "device" pointers are HIP device
 *     memory on the context's device, "host" pointers are ordinary memory.
 *   - Dense matrices are row-major.  K is symmetric; only its lower triangle
 *     (i >= j) is read, and the factor overwrites the strict lower triangle
 *     with L (unit diagonal implicit) -- row-major lower == the reference's
 *     L[i][j], i > j.
 *   - Return value: 0 success; > 0 = 1-based index of the first non-finite
 *     pivot (the factorization still completes, as the reference's does);
 *     < 0 = error (IPMZ_ERR_*), message via ipmz_last_error().  The zero-pivot
 *     rule of the reference (an exactly-zero pivot becomes 1e-8,
 *     LinearSolvers.cpp:26-28) is not an error, as in the reference.
 *   - All device work is enqueued on the context's stream; functions whose
 *     outputs are host memory synchronize it.
 *   - There is no CPU fallback: without a usable gfx950 device every entry
 *     point that computes returns IPMZ_ERR_NO_DEVICE.
 */
#ifndef IPMZ_H
#define IPMZ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IPMZ_OK 0
#define IPMZ_ERR_INVALID (-1)
#define IPMZ_ERR_HIP (-2)
#define IPMZ_ERR_NOMEM (-3)
#define IPMZ_ERR_NO_DEVICE (-4)
#define IPMZ_ERR_STATE (-5)

/* Canonical Newton-variable slots.  The reference's Newton-variable order
 * (get_newton_system, SlackedSlacks + Regularization) is this order with the
 * absent blocks dropped; state vectors are concatenated in it. */
enum ipmz_slot {
  IPMZ_SLOT_X = 0, IPMZ_SLOT_LAMBDA_A, IPMZ_SLOT_LAMBDA_C, IPMZ_SLOT_S, IPMZ_SLOT_P,
  IPMZ_SLOT_LAMBDA_G, IPMZ_SLOT_LAMBDA_H, IPMZ_SLOT_LAMBDA_Y, IPMZ_SLOT_LAMBDA_Z,
  IPMZ_SLOT_G, IPMZ_SLOT_H, IPMZ_SLOT_Y, IPMZ_SLOT_Z, IPMZ_NSLOT
};

/* Per-iteration scalars (device block of IPMZ_SC_COUNT doubles). */
enum ipmz_scalar {
  IPMZ_SC_F = 0,        /* objective 0.5 x'Qx + c'x of the current iterate   */
  IPMZ_SC_RES,          /* ||full rhs at mu = 0||_2 (get_residual_norm_)      */
  IPMZ_SC_MU,           /* mean |complementarity| (get_mu_)                   */
  IPMZ_SC_ALPHA_AFF,    /* last step: affine step length                      */
  IPMZ_SC_MU_AFF,       /* last step: mu at the affine trial point            */
  IPMZ_SC_SIGMA,        /* last step: (mu_aff / mu)^3                         */
  IPMZ_SC_ALPHA,        /* last step: corrector step length (before 0.995)    */
  IPMZ_SC_CONVERGED,    /* 1.0 when res < 1e-8 and mu < 1e-8                  */
  IPMZ_SC_MU_NEW,       /* last step: sigma * mu                              */
  IPMZ_SC_RESTARTS,     /* benchmark restarts taken                           */
  IPMZ_SC_IR_RATIO_AFF, /* mixed precision: ||r||/||b|| reached, affine solve */
  IPMZ_SC_IR_ITERS_AFF, /*   refinement corrections, affine solve             */
  IPMZ_SC_IR_RATIO,     /*   the same for the corrector solve                 */
  IPMZ_SC_IR_ITERS,
  IPMZ_SC_COUNT = 16
};

typedef struct ipmz_ctx ipmz_ctx;
typedef struct ipmz_qp ipmz_qp;

/* ---- context ---------------------------------------------------------- */
int ipmz_ctx_create(ipmz_ctx** out, int device);
/* Destroying a context that solvers (ipmz_qp_create / ipmz_batch_create)
 * still use only marks it: it is freed when the last of them is destroyed
 * (so a garbage collector may finalize the two in either order; the calls
 * are thread-safe with respect to each other).  A marked context first
 * drains an external stream set with ipmz_ctx_set_stream and then runs its
 * remaining solvers on its own stream; creating a solver on it returns
 * IPMZ_ERR_STATE. */
int ipmz_ctx_destroy(ipmz_ctx* ctx);
/* Enqueue on an external HIP stream, e.g. torch.cuda.current_stream().cuda_stream.
 * NULL selects the HIP null (legacy default) stream -- what PyTorch's
 * default stream is -- NOT the context's own stream. */
int ipmz_ctx_set_stream(ipmz_ctx* ctx, void* hip_stream);
/* Go back to the context's own (non-blocking) stream. */
int ipmz_ctx_reset_stream(ipmz_ctx* ctx);
int ipmz_ctx_sync(ipmz_ctx* ctx);
const char* ipmz_last_error(void);
/* Test hook: while bit 1 (solve) / bit 2 (outer-panel factor) is set, the
 * persistent kernels launched drop their first cross-workgroup hand-off, so
 * their consumers hit the 0.5 s spin limit -- the path by which a stuck
 * hand-off surfaces as IPMZ_ERR_HIP from ipmz_ldlt_factor, ipmz_ctx_sync,
 * ipmz_qp_scalars, ipmz_qp_solve (sticky error words, cleared when a
 * factorization starts).  Bit 4 is not a fault: IPMZ_STEP_GRAPH then
 * captures steps whose factor forks onto the look-ahead streams as well.
 * 0 (default) for normal operation. */
int ipmz_debug_inject(int mask);
/* Blocking of the factorization: outer panel nbo (multiple of nbi, <= 512;
 * 0 = by matrix order: with nbi 64, 512 for N > 4096, 384 for 2048 <= N <= 4096,
 * else 256), inner
 * diagonal block nbi (64 or 128).  Defaults 0 / 64.  Workspace sizes depend
 * on it: query them after setting the blocking. */
int ipmz_ctx_set_blocking(ipmz_ctx* ctx, int nbo, int nbi);
/* The blocking an order-N factor uses with this context (nbo resolved when
 * the context's is 0 = by matrix order). */
int ipmz_ctx_get_blocking(ipmz_ctx* ctx, int N, int* nbo, int* nbi);

/* ---- LinearSolvers on device memory ------------------------------------ */
/* Workspace for factor + solve of order N (bytes). */
int64_t ipmz_ldlt_workspace_bytes(ipmz_ctx* ctx, int N);
/* In-place LDL^T of the lower triangle of K (device, row-major, ld >= N,
 * ld even).  D: device, N doubles.  ws: device workspace; it keeps the
 * inverted diagonal blocks that ipmz_ldlt_solve consumes. */
int ipmz_ldlt_factor(ipmz_ctx* ctx, int N, double* K, int64_t ld, double* D, void* ws, int64_t ws_bytes);
/* b <- K^{-1} b with the factor left by ipmz_ldlt_factor (device b); asynchronous.
 * ws must stay allocated until the next ipmz_ctx_sync, which reports a
 * hand-off timeout of this solve (its sticky error words) as IPMZ_ERR_HIP. */
int ipmz_ldlt_solve(ipmz_ctx* ctx, int N, const double* K, int64_t ld, const double* D, const void* ws, double* b);
/* Rebuild the solve workspace from an explicit unit-lower L (device). */
int ipmz_ldlt_prepare_solve(ipmz_ctx* ctx, int N, const double* L, int64_t ld, void* ws, int64_t ws_bytes);

/* ---- mixed precision (config C5): fp32 factor + fp64 refinement -----------
 * No reference counterpart (the reference is fp64 throughout,
 * LinearSolvers.cpp:14-74); the result is the fp64 solution of the same
 * system to the requested tolerance.  K: device, lower triangle, row-major,
 * fp64 (left intact: the refinement residual r = b - K x uses it).  The
 * factor is of S K S, S = diag(|K_ii|^-1/2), stored in fp32 in ws. */
int64_t ipmz_mixed_workspace_bytes(ipmz_ctx* ctx, int N);
int ipmz_mixed_factor(ipmz_ctx* ctx, int N, const double* K, int64_t ld, void* ws, int64_t ws_bytes);
/* b (device) <- K^{-1} b, refined until ||b - K x||_inf <= tol ||b||_inf or
 * max_refine corrections; stat (host, may be NULL): {ratio reached,
 * corrections applied}. */
int ipmz_mixed_solve(ipmz_ctx* ctx, int N, const double* K, int64_t ld, void* ws, double* b, double tol,
                     int max_refine, double* stat);

/* ---- normal-equations reduction (config C2) ------------------------------
 * The reference derives it symbolically (get_normal_equations,
 * SymbolicOptimization.cpp:465-478; built at Optimizer.cpp:39-40) but never
 * evaluates it.  For the augmented K = [[H, B^T], [B, -E]] (device, lower
 * triangle, order n + mp, H SPD, E > 0 diagonal): Cholesky of H (as L D L^T,
 * D > 0), L21 = B L^{-T} D^{-1}, S = E + L21 D L21^T = E + B H^{-1} B^T,
 * Cholesky of S -- run as the x-first blocked LDL^T of K, one pipelined
 * factor (normal.hip).  K's lower triangle is overwritten by [L_H; L21, L_S].
 * D: device, n + mp doubles (pivots of H, then of -S).  Returns > 0 (1-based
 * augmented index) when H or S is not positive definite. */
int64_t ipmz_normal_workspace_bytes(ipmz_ctx* ctx, int n, int mp);
int ipmz_normal_factor(ipmz_ctx* ctx, int n, int mp, double* K, int64_t ld, double* D, void* ws, int64_t ws_bytes);
/* b = [r0; r1] (device) <- [x; l]:  l = S^{-1} (B H^{-1} r0 - r1),
 * x = H^{-1} (r0 - B^T l). */
int ipmz_normal_solve(ipmz_ctx* ctx, int n, int mp, const double* K, int64_t ld, const double* D, void* ws, double* b);

/* ---- Bunch-Kaufman (symmetric indefinite) ---------
 * LinearSolvers::symmetric_indefinite_factorization (LinearSolvers.h:23-26,
 * LinearSolvers.cpp:76-207) and overwriting_solve_bunch_kaufman
 * (LinearSolvers.h:28-31, :209-318); never called by the reference's
 * Optimizer (solve_indefinite_ is ASSERT(false), Optimizer.cpp:75).
 * Device: A row-major (lower triangle factored in place), any N; ipiv:
 * device int[N] in the reference's convention (>= 0: 1x1 pivot with that
 * interchange; < 0: -kp on both rows of a 2x2 pivot).  fix_kp = 0 keeps the
 * reference's kp = 0 for a second all-zero column (LinearSolvers.cpp:111-116),
 * 1 records kp = k.  Returns 0, or 1 + the first all-zero column. */
int ipmz_bk_factor(ipmz_ctx* ctx, int N, double* A, int64_t ld, int* ipiv, int fix_kp);
/* Same, with the kernel chosen: IPMZ_BK_AUTO (the whole-device factor from
 * N = 512 up), IPMZ_BK_WORKGROUP (one workgroup, N <= 4096), IPMZ_BK_GRID
 * (every CU, a grid barrier per pivot step).  Both are bitwise the reference. */
#define IPMZ_BK_AUTO 0
#define IPMZ_BK_WORKGROUP 1
#define IPMZ_BK_GRID 2
int ipmz_bk_factor_ex(ipmz_ctx* ctx, int N, double* A, int64_t ld, int* ipiv, int fix_kp, int algo);
/* b <- A^{-1} b from ipmz_bk_factor's F and ipiv, in the reference's order
 * (overwriting_solve_bunch_kaufman, LinearSolvers.cpp:209-318).  From
 * N = 512 it reads a transposed copy of F made on the context's stream
 * (N * N doubles, stream-ordered allocation freed after the solve). */
int ipmz_bk_solve(ipmz_ctx* ctx, int N, const double* F, int64_t ld, const int* ipiv, double* b);
/* Host signatures of the reference (value semantics, reference pivoting
 * including its kp = 0 defect): F = A with the lower triangle factored. */
int ipmz_symmetric_indefinite_factorization(ipmz_ctx* ctx, int N, const double* A, double* F, int* ipiv);
int ipmz_overwriting_solve_bunch_kaufman(ipmz_ctx* ctx, int N, const double* F, const int* ipiv, double* b);

/* ---- LinearSolvers with the reference's host signatures ------------------ */
/* A: host N x N row-major (lower triangle read).  L: host N x N, written
 * full (zeros above, ones on the diagonal); D: host N. */
int ipmz_ldlt_decomposition(ipmz_ctx* ctx, int N, const double* A, double* L, double* D);
/* L: host N x N unit lower; D: host N; b: host N, overwritten with the
 * solution.  N == 0 is a no-op (LinearSolvers.cpp:46-48). */
int ipmz_overwriting_solve_ldlt(ipmz_ctx* ctx, int N, const double* L, const double* D, double* b);

/* ---- the Newton-step solver --------------------------------------------- */
/* Settings::EqualityHandling (SymbolicOptimization.h:28-64) */
#define IPMZ_EQ_REGULARIZATION 0 /* (lambda_C, lambda_C) block -delta^2, slack p: LDL^T   */
#define IPMZ_EQ_NONE 1           /* zero (lambda_C, lambda_C) block, no p: the reference's
                                    "indefinite" case (Optimizer.cpp:63-75), factored with
                                    Bunch-Kaufman (LinearSolvers.cpp:76-318): any N for a
                                    single QP (the whole-device factor from N = 512), N <= 4096
                                    per QP in batches (one workgroup per QP) */
#define IPMZ_EQ_PENALTY 2        /* PenaltyFunction: -mu (lambda_C, lambda_C) block (mu I,
                                    mu = the iterate's environment mu), no p: LDL^T */
#define IPMZ_EQ_PENALTY_EXTRA_DUAL 3 /* PenaltyFunctionWithExtraDual: the reference derives
                                        PenaltyFunction's optimality conditions through it
                                        (SymbolicOptimization.cpp:364-366) -- the same Newton
                                        system (tests/golden/formulations.txt), solved alike */
#define IPMZ_EQ_SLACKED_SLACKS 4 /* equality SlackedSlacks: t with slacks v = t - d, w = d - t
                                    (l = u = d), their duals lambda_v, lambda_w; the KKT
                                    (lambda_C, lambda_C) block -((V^-1 L_v) + (W^-1 L_w))^-1.
                                    With InequalityHandling::SlackedSlacks and both
                                    inequality bounds; the reference's evaluator asserts
                                    on its zero blocks (Evaluation.cpp:57-60) */
#define IPMZ_EQ_NAIVE_SLACKS 5   /* equality NaiveSlacks: C x - v = d, C x + w = d with duals
                                    lambda_v, lambda_w as KKT rows (SymbolicOptimization.cpp:
                                    163-171; N = n + 2m + 2p).  With InequalityHandling::
                                    NaiveSlacks and both inequality bounds: the rows run as
                                    NaiveSlacks inequality rows with l = u = d */
/* Settings::InequalityHandling (SymbolicOptimization.h:28-64) */
#define IPMZ_INEQ_SLACKED_SLACKS 0 /* s with slacks g = s - l_A, h = u_A - s (and y, z
                                      for x): the reference default                  */
#define IPMZ_INEQ_SLACKS 1         /* no g/h/y/z: complementarity on (s - l_A) lambda_g
                                      etc.; the reference's corrector substitutes
                                      dX_aff for X in (X - L_x),
                                      reproduced.  Bounds must be IPMZ_BOUNDS_BOTH
                                      (inequality bounds: when m > 0). */
#define IPMZ_INEQ_NAIVE_SLACKS 2   /* no s: l_A + g = A x, A x + h = u_A with duals lambda_g,
                                      lambda_h as KKT rows (N = n + 2m + p); the reference's
                                      evaluator asserts on its zero block, Evaluation.cpp:
                                      57-60.  Both inequality bounds; not with the
                                      normal-equations reduction. */
/* Settings::Bounds for inequality_bounds / variable_bounds */
#define IPMZ_BOUNDS_BOTH 0
#define IPMZ_BOUNDS_LOWER 1
#define IPMZ_BOUNDS_UPPER 2
#define IPMZ_BOUNDS_NONE 3 /* variable bounds only; inequalities need a bound when m > 0 */
typedef struct ipmz_qp_config {
  int n;         /* primal dimension                                  */
  int m;         /* inequality rows  l_A <= A x <= u_A                 */
  int p;         /* equality rows C x = d                              */
  double delta;  /* regularization (EnvironmentBuilder.cpp:48: 1e-4)  */
  int equality_handling;   /* IPMZ_EQ_* (0 = Regularization)          */
  int inequality_handling; /* IPMZ_INEQ_* (0 = SlackedSlacks)         */
  int inequality_bounds;   /* IPMZ_BOUNDS_* (0 = Both)                */
  int variable_bounds;     /* IPMZ_BOUNDS_* (0 = Both)                */
} ipmz_qp_config;

int ipmz_qp_create(ipmz_ctx* ctx, const ipmz_qp_config* cfg, ipmz_qp** out);
int ipmz_qp_destroy(ipmz_qp* qp);
/* build_environment: validates l_x < u_x and l_A <= u_A (throws in the
 * reference, IPMZ_ERR_INVALID here), copies the data, sets the initial
 * iterate and evaluates it.  Host pointers; unused blocks may be NULL. */
int ipmz_qp_load_host(ipmz_qp* qp, const double* Q, const double* c, const double* A, const double* l_A,
                      const double* u_A, const double* C, const double* d, const double* l_x, const double* u_x);
/* The synthetic QP of SURVEY.md §8d generated in place on the device. */
int ipmz_qp_generate(ipmz_qp* qp, uint64_t seed);
/* Enqueue one Newton step (asynchronous).  A step whose factor forks onto the
 * look-ahead streams (>= 3 outer panels) is kept to one in flight: on the
 * context's own stream the next call waits for it; on a stream set with
 * ipmz_ctx_set_stream it runs on the context's own stream and the call
 * returns once it completed, the caller's stream joined to it (a join left
 * pending on the caller's stream slows the step).  A step
 * through the mixed-precision solve (ipmz_qp_set_mixed_precision) also
 * blocks the host while its refinement runs: the eager loop reads a
 * host-mapped stop test after each pass instead of enqueuing all
 * max_refine + 1 passes.  When the caller's stream is capturing a hipGraph
 * the step is enqueued into that capture on that stream (no host wait, all
 * refinement passes, IPMZ_STEP_GRAPH ignored).  flags: */
#define IPMZ_STEP_RESTART_IF_CONVERGED 1 /* reset a converged iterate to the initial one first */
#define IPMZ_STEP_GRAPH 2                /* capture once into a hipGraph, then replay (steps whose
                                            factor forks onto the look-ahead streams -- >= 3 outer
                                            panels -- are enqueued eagerly instead) */
int ipmz_qp_step(ipmz_qp* qp, int flags);
/* 1 when the last ipmz_qp_step replayed a captured hipGraph, 0 when its
 * launches were enqueued one by one (what a benchmark reports it timed). */
int ipmz_qp_last_step_graph(ipmz_qp* qp);
/* Synchronize and copy the IPMZ_SC_COUNT scalars to host memory. */
int ipmz_qp_scalars(ipmz_qp* qp, double* out);
/* Device pointer of the scalar block (for collectives). */
int ipmz_qp_device_scalars(ipmz_qp* qp, double** out);
/* Enqueue a device-to-device copy of the scalar block to dst (device). */
int ipmz_qp_copy_scalars(ipmz_qp* qp, double* dst_device);
/* Optimizer::solve: iterate until res < 1e-8 and mu < 1e-8 or max_iter.
 * trace (host, may be NULL): max_iter rows of 8 doubles
 * {f, res, mu, alpha_aff, mu_aff, sigma, alpha, converged}. */
int ipmz_qp_solve(ipmz_qp* qp, int max_iter, double* trace, int* iterations);
/* Concatenated state in Newton order.  which: 0 iterate, 1 affine
 * direction, 2 corrector direction, 3 residual vectors r_v. */
#define IPMZ_STATE_VARS 0
#define IPMZ_STATE_DAFF 1
#define IPMZ_STATE_DIR 2
#define IPMZ_STATE_RES 3
int64_t ipmz_qp_state_len(ipmz_qp* qp);
int ipmz_qp_get_state(ipmz_qp* qp, int which, double* host_out);
/* Overwrite the iterate (host, Newton order) and re-evaluate it. */
int ipmz_qp_set_state(ipmz_qp* qp, const double* host_vars);
/* Assemble the KKT matrix of the current iterate; host N x N row-major
 * (lower triangle written, upper zero).  For parity tests. */
int ipmz_qp_get_kkt(ipmz_qp* qp, double* host_K);
int ipmz_qp_kkt_dim(ipmz_qp* qp);
/* Newton directions through the mixed-precision solve (fp32 factor of the
 * scaled KKT matrix + fp64 refinement to tol, at most max_refine corrections
 * per solve); enable = 0 returns to the fp64 factor.  Single QPs only.  The
 * scalar block then reports IPMZ_SC_IR_*. */
int ipmz_qp_set_mixed_precision(ipmz_qp* qp, int enable, double tol, int max_refine);
/* KKT reduction of the Newton step: augmented LDL^T (default, what the
 * reference solves, Optimizer.cpp:137-138) or the normal equations (the
 * reference's normal_equations_ reduction, Optimizer.cpp:39-40).  Single
 * QPs; not combined with mixed precision. */
#define IPMZ_REDUCTION_AUGMENTED 0
#define IPMZ_REDUCTION_NORMAL 1
int ipmz_qp_set_reduction(ipmz_qp* qp, int reduction);

/* ---- batches of independent QPs (config C4) ------------------------------
 * A batch is an ipmz_qp holding `batch` QPs of identical (n, m, p); every
 * kernel launch serves the whole batch.  ipmz_qp_step / _generate (QP i gets
 * seed + i) / _destroy / _set_timing / _phase_times apply to batches; the
 * ipmz_qp_* state accessors address QP 0. */
int ipmz_batch_create(ipmz_ctx* ctx, const ipmz_qp_config* cfg, int batch, ipmz_qp** out);
int ipmz_batch_size(ipmz_qp* qp);
/* Copy QP `index`'s data (build_environment's validation); call
 * ipmz_batch_initialize once every QP is loaded.  A load leaves the batch
 * uninitialized: ipmz_qp_step / ipmz_batch_solve return IPMZ_ERR_STATE until
 * ipmz_batch_initialize has rebuilt the kept KKT matrix and the residuals
 * from the new data (a step on the previous data's matrix would be silent
 * corruption). */
int ipmz_batch_load_host(ipmz_qp* qp, int index, const double* Q, const double* c, const double* A,
                         const double* l_A, const double* u_A, const double* C, const double* d, const double* l_x,
                         const double* u_x);
int ipmz_batch_initialize(ipmz_qp* qp);
/* out: host, batch * IPMZ_SC_COUNT doubles */
int ipmz_batch_scalars(ipmz_qp* qp, double* out);
int ipmz_batch_get_state(ipmz_qp* qp, int index, int which, double* host_out);
int ipmz_batch_set_state(ipmz_qp* qp, int index, const double* host_vars);
/* Enqueue a device-to-device copy of all batch * IPMZ_SC_COUNT scalars
 * (QP-major) to dst (device): the input of the cross-GPU convergence summary. */
int ipmz_batch_copy_scalars(ipmz_qp* qp, double* dst_device);
/* Enqueue ONE kernel writing the batch's convergence summary to dst (device,
 * 3 doubles): {max res, max mu, unconverged count} over its QPs -- the
 * stopping rule of Optimizer.cpp:124-135 in MAX-reducible form, so a single
 * all-reduce (MAX) across the ranks of a sharded batch decides the stop
 * (reduced dst[2] == 0 <=> every QP of the job converged).  For the RCCL
 * driver loop of ipmz_amd.dist.solve_sharded. */
int ipmz_batch_summary(ipmz_qp* qp, double* dst_device);
/* Step until every QP converged (converged QPs keep their iterate). */
int ipmz_batch_solve(ipmz_qp* qp, int max_iter, int* iterations, int* converged_count);
/* Which kernel factors a batch of small systems (N <= 1024, 64-column
 * blocks, one LDL^T): IPMZ_BATCH_FACTOR_AUTO (default: the wave-specialized
 * left-looking kernel for 64 < N <= 320; above that two workgroups per QP
 * when 2 * batch <= #CU, else the left-looking one), IPMZ_BATCH_FACTOR_ONE
 * (right-looking, one workgroup per QP), IPMZ_BATCH_FACTOR_PAIR (the same
 * right-looking factor on two workgroups per QP -- identical results to ONE;
 * IPMZ_ERR_INVALID unless 2 * batch <= #CU, since both workgroups of a QP
 * must be resident together), IPMZ_BATCH_FACTOR_LEFT (left-looking, one
 * workgroup per QP: every L tile formed once in registers; sums in a
 * different order, so 1e-16-level differences against ONE / PAIR). */
#define IPMZ_BATCH_FACTOR_AUTO 0
#define IPMZ_BATCH_FACTOR_ONE 1
#define IPMZ_BATCH_FACTOR_PAIR 2
#define IPMZ_BATCH_FACTOR_LEFT 3
int ipmz_batch_set_factor_kernel(ipmz_qp* qp, int kernel);

/* Phase timing (HIP events on the context stream; eager launches only).
 * ms: host array of IPMZ_PH_COUNT floats, cumulative since enable. */
enum ipmz_phase {
  IPMZ_PH_STEP = 0, IPMZ_PH_ASSEMBLE, IPMZ_PH_FACTOR, IPMZ_PH_SOLVE, IPMZ_PH_TRAILING, IPMZ_PH_EVAL,
  IPMZ_PH_COUNT = 8
};
int ipmz_qp_set_timing(ipmz_qp* qp, int enable);
int ipmz_qp_phase_times(ipmz_qp* qp, double* ms, double* trailing_flops, int64_t* trailing_launches);

#ifdef __cplusplus
}
#endif
#endif /* IPMZ_H */
