// Host-side launchers of the gfx950 kernels (internal to libipmz).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define IPMZ_NBO_MAX 512
#define IPMZ_PANEL_CTRL_WORDS 320
// fused factor: largest N whose chain launches start beside the previous
// panel's rows launch (ldlt.hip)
#define IPMZ_EARLY_CHAIN_MAX_N 4096
// rows per partial sum of the transposed mat-vecs A^T y, C^T y (newton.hip)
#define IPMZ_TCHUNK 32
#define IPMZ_CHAIN_STAMP_BLOCKS 512  // (debug stamps: N <= 32768)
#define IPMZ_SOLVE_BLOCK 128     // rows per block of the persistent solve
#define IPMZ_SOLVE_CTRL_WORDS 8  // its control words (error, tickets, sweep counters)

namespace ipmz {

// Fault injection for the tests of the spin-timeout path (ipmz_debug_inject):
// a persistent kernel launched while its bit is set drops its first
// hand-off, so every consumer times out and raises the sticky error word.
// IPMZ_INJECT_GRAPH_FORKS: not a fault -- IPMZ_STEP_GRAPH captures steps whose
// factor forks onto the look-ahead streams too (the capture experiment of
// tests/test_gpu_graph.py, bitwise the eager step) instead of enqueuing them
// eagerly (the production choice: graph replay of a forked step is slower).
// DEBUG bits (determinism experiments): 16 = the mixed factor stops after
// the scale + fp32 conversion, 32 = factors run on one stream (no look-ahead)
// 64 = trace the host calls of a step to stderr (the capture experiment),
// 128 = the fp32 trailing and strip updates on the gemm.h engine instead of gemm32.h (A/B),
// 256 = the fp32 factor's look-ahead strip on the trailing stream before the trailing update (no fourth stream),
// 512 = the eager mixed-precision solve enqueues all max_refine + 1 passes (no host stop test),
// 1024 = the fp64 trailing and strip updates on gemm.h's register-staged kernel instead of gemm64.h's (A/B),
// 2048 = an early chain launch (started beside the previous panel's rows launch) never sees that
//        launch's RDONE flags: it gives its roles back after 1 ms and the rows launch takes them
//        (the serialized-dispatch path, tests/test_gpu_panel_forms.py),
// 4096 = the chain launch draws no ticket: the rows launch runs every chain role in its 4-wave form
//        (what a serialized dispatch order can produce; the forms must factor bitwise alike),
// 8192 = batches assemble the whole KKT into K every step (not the kept K0) (A/B),
// 16384 = batches run the two solves and the phases between them as separate launches (A/B)
enum { IPMZ_INJECT_SOLVE = 1, IPMZ_INJECT_PANEL = 2, IPMZ_INJECT_GRAPH_FORKS = 4, IPMZ_DEBUG_CONVERT_ONLY = 16,
       IPMZ_DEBUG_ONE_STREAM = 32, IPMZ_DEBUG_TRACE = 64, IPMZ_DEBUG_F32_ENGINE = 128,
       IPMZ_DEBUG_NO_FOURTH = 256, IPMZ_DEBUG_IR_FULL = 512,
       IPMZ_DEBUG_F64_ENGINE = 1024, IPMZ_DEBUG_GIVEBACK = 2048, IPMZ_DEBUG_ROWS_CHAIN = 4096,
       IPMZ_DEBUG_NO_K0 = 8192, IPMZ_DEBUG_NO_FUSED_SOLVES = 16384, IPMZ_DEBUG_READY_LATE = 32768 };
#define IPMZ_TRACE(...)                                                  \
  do {                                                                   \
    if (::ipmz::debug_inject_mask() & ::ipmz::IPMZ_DEBUG_TRACE) {        \
      fprintf(stderr, "[ipmz] " __VA_ARGS__);                            \
      fputc('\n', stderr);                                              \
      fflush(stderr);                                                    \
    }                                                                    \
  } while (0)
int debug_inject_mask();
// cross-stream ordering that a capture on the HIP runtime torch bundles can
// end (ldlt.hip): event records / waits of the factor's look-ahead streams
hipError_t stream_record(hipEvent_t e, hipStream_t s);
hipError_t stream_wait(hipStream_t s, hipEvent_t e);
void set_capture_origin(hipStream_t s);  // the stream a capture began on (nullptr: none)
void set_debug_inject_mask(int mask);
// error words the persistent kernels raise on a spin timeout (sync.h): the
// panel kernel's ctrl[PANEL_ERR_WORD], the solve's ctrl[1]
constexpr int PANEL_ERR_WORD = 2;
constexpr int SOLVE_ERR_WORD = 1;

// ldlt.hip -------------------------------------------------------------------
// Batched factorization: element strides between consecutive QPs' K, D,
// L^{-1} blocks and W panels.
struct BatchStrides {
  int B = 1;
  int64_t sK = 0, sD = 0, sL = 0, sW = 0;
  // small batched factor: B * IPMZ_PAIR_FLAGS + 1 words for the two-workgroup
  // factor (B <= #CU; W then needs 2 x N x 64 per QP), nullptr = one workgroup
  unsigned* pflags = nullptr;
  // small batched factor: the assembled KKT's first touch (block column 0's
  // steps) read from K0 (strides sK) instead of K -- the off-diagonal part
  // kept across Newton steps, only its diagonal rewritten per step; nullptr =
  // K holds the assembled matrix
  const double* K0 = nullptr;
  // small batched factor: IPMZ_BATCH_FACTOR_* (ipmz.h)
  int small_kernel = 0;
};
#define IPMZ_PAIR_FLAGS 32  // per QP: LW[16], DONE[16] (N <= IPMZ_SMALL_NMAX)
// the batched factor of order N runs two workgroups per QP (given flags)
bool small_pair_eligible(int B, int N);
bool small_pair_used(int kern, bool have_flags, int B, int N);
// small.hip: whole factor per workgroup (N <= IPMZ_SMALL_NMAX, nbi = 64;
// W: N x 64 per QP)
#define IPMZ_SMALL_NMAX 1024
hipError_t ldlt_factor_small_batched(double* K, int64_t ld, int N, double* D, double* Linv, double* W, int* info,
                                     hipStream_t st, const BatchStrides& bs);
hipError_t ldlt_factor_small_variant(int snw, double* K, int64_t ld, int N, double* D, double* Linv, double* W,
                                     int* info, hipStream_t st, const BatchStrides& bs);  // kbench only
hipError_t ldlt_factor_batched(double* K, int64_t ld, int N, double* D, double* Linv, double* W, int nbo, int nbi,
                               int* info, hipStream_t st, const BatchStrides& bs);
// In-place blocked LDL^T of the lower triangle of K (row-major, ld).
// Linv: (ceil(N/nbi)) blocks of nbi x nbi (inverse unit-lower diagonal
// blocks, consumed by ldlt_solve); W: N x nbo workspace.  info: device int,
// preset to INT_MAX-ish; receives min(1-based index of a non-finite pivot).
// trailing updates of order <= this run on 64 x 64 tiles, larger ones on the
// 128 x 128 kernel (the one TrailTimer times: the roofline kernel of bench.py)
#define IPMZ_TRAIL_SMALL_M 3072
struct TrailTimer {  // HIP-event pairs around every dominant trailing-update launch
  hipEvent_t (*pairs)[2] = nullptr;
  int cap = 0, used = 0;
  double flops = 0.0;
  hipEvent_t* next() { return used < cap ? pairs[used++] : nullptr; }
};
// Look-ahead when st2 (and, for the panel path, st3) and ev (>= 4 *
// ceil(N/nbo) + 2 events) are given; W must then hold 3 * N * nbo doubles
// (else N * nbo).  pctrl: panel_ctrl_words(N, nbo) zeroed words for the
// panel path of panel.hip (nbi == 64); nullptr selects the diag / TRSM /
// strip kernel chain.
hipError_t ldlt_factor(double* K, int64_t ld, int N, double* D, double* Linv, double* W, int nbo, int nbi,
                       int* info, hipStream_t st, TrailTimer* timer = nullptr, hipStream_t st2 = nullptr,
                       hipStream_t st3 = nullptr, hipEvent_t* ev = nullptr, int nev = 0, unsigned* pctrl = nullptr, hipStream_t st4 = nullptr);
// the same blocked LDL^T in fp32 (fp32 MFMA trailing update): the factor of
// the mixed-precision solve (C5)
hipError_t ldlt_factor(float* K, int64_t ld, int N, float* D, float* Linv, float* W, int nbo, int nbi, int* info,
                       hipStream_t st, TrailTimer* timer, hipStream_t st2, hipStream_t st3, hipEvent_t* ev, int nev,
                       unsigned* pctrl = nullptr, hipStream_t st4 = nullptr);
// ctrl words of the panel path: a shared area (sticky error word) + one
// area per outer panel, then three 64 x 64 (8-byte) tiles: the next panel's
// block (0, 0) look-ahead update, pre-accumulated by the rows launch (three,
// so a rows launch never waits for the chain launch that read the slot it
// reuses)
#define IPMZ_PANEL_PRE00_WORDS (3 * 64 * 64 * 2)
inline int64_t panel_ctrl_words(int N, int nbo) {
  return (int64_t)IPMZ_PANEL_CTRL_WORDS * (1 + (N + nbo - 1) / nbo) + IPMZ_PANEL_PRE00_WORDS;
}
// one outer panel [k0, k0 + bo) of the panel path (panel.hip): the chain
// launch on st_chain, the rows launch on st_rows (flags in `area`, sticky
// error word `err`).  Lb0: L^{-1} block of the panel's first inner block; Wp:
// the panel's W buffer (N x ldw, row-indexed).  Wprev != nullptr: the chain
// launch first applies the look-ahead update with the previous panel
// [kprev, kprev + boprev) (W_prev rows, ld ldw) to the panel's diagonal
// region (and, rows_prev, the rows launch to its rows).
hipError_t panel_factor(double* K, int64_t ld, int N, int k0, int bo, double* D, double* Lb0, double* Wp, int ldw,
                        const double* pre00_in, double* pre00_out,
                        int* info, unsigned* area, unsigned* err, const double* Wprev, int kprev, int boprev,
                        bool rows_prev, hipStream_t st_chain, hipStream_t st_rows,
                        const unsigned* parea = nullptr, bool wait_ready = false);
hipError_t panel_factor(float* K, int64_t ld, int N, int k0, int bo, float* D, float* Lb0, float* Wp, int ldw,
                        const float* pre00_in, float* pre00_out,
                        int* info, unsigned* area, unsigned* err, const float* Wprev, int kprev, int boprev,
                        bool rows_prev, hipStream_t st_chain, hipStream_t st_rows,
                        const unsigned* parea = nullptr, bool wait_ready = false);
// wait_ready: the chain roles of the panel's chain launch first wait for the
// panel's READY-TO-FACTOR word, raised by panel_ready on the stream of the
// look-ahead update the panel's columns needed last (instead of a
// cross-stream wait before that launch), then acquire (agent scope)
hipError_t panel_ready(unsigned* area, hipStream_t st);
hipError_t linv_from_l(const double* L, int64_t ld, int N, int nbi, double* Linv, hipStream_t st);
hipError_t gemm_nt_sub(int M, int N, int Kd, const double* A, int64_t lda, const double* B, int64_t ldb,
                       double* C, int64_t ldc, int64_t row0, int64_t col0, bool square_lower, hipStream_t st,
                       const BatchStrides* bs = nullptr);

// trsv.hip -------------------------------------------------------------------
// In-place b <- L^{-T} D^{-1} L^{-1} b; side: 2*nbi doubles of scratch.
hipError_t ldlt_solve(const double* K, int64_t ld, int N, const double* D, const double* Linv, int nbi, double* b,
                      double* side, hipStream_t st);

// one workgroup per QP of a batch (small N); b: batch of rhs, stride sb
hipError_t ldlt_solve_batched(const double* K, int64_t ld, int N, const double* D, const double* Linv, int nbi,
                              double* b, int B, int64_t sK, int64_t sD, int64_t sL, int64_t sb, hipStream_t st);

// trsv_persist.hip: the same solve as ONE persistent launch on 128-row
// blocks (nbi == 64 factors).  P: solve_prep_elems(N) elements written by
// solve_prep from the factor's 64 x 64 inverses (once per factorization);
// ybuf, xbuf: N elements; ctrl: IPMZ_SOLVE_CTRL_WORDS unsigned, all set up
// by solve_reset once per factorization (ctrl[SOLVE_ERR_WORD] is sticky).
int64_t solve_prep_elems(int N);
// the persistent solve's state after a factorization: control words zero,
// y / x buffers (N elements of size elem) all-ones sentinels; the solve
// launches keep it so for the next solve.  Optionally in the same launch:
// info / info2 words set to 0x7f7f7f7f ("no failed pivot") and nwords words
// zeroed (a factor's panel ctrl words)
hipError_t solve_reset(void* ybuf, void* xbuf, size_t elem, int N, unsigned* ctrl, hipStream_t st,
                       int* info = nullptr, unsigned* words = nullptr, int64_t nwords = 0, int* info2 = nullptr);
hipError_t solve_stamps(unsigned long long* out);  // DEBUG
hipError_t chain_stamps(unsigned long long* c, unsigned long long* h);  // DEBUG (-DIPMZ_CHAIN_STAMPS)
hipError_t solve_prep(const double* K, int64_t ld, int N, const double* Linv, double* P, hipStream_t st);
hipError_t solve_prep(const float* K, int64_t ld, int N, const float* Linv, float* P, hipStream_t st);
hipError_t ldlt_solve_persistent(const double* K, int64_t ld, int N, const double* D, const double* P, double* b,
                                 double* ybuf, double* xbuf, unsigned* ctrl, hipStream_t st);
// one sweep (forward: ybuf = L^{-1} b; backward: b = L^{-T} (ybuf / D)); skip
// (device flag, may be null): return at once when set
hipError_t ldlt_solve_persistent_sweep(const double* K, int64_t ld, int N, const double* D, const double* P,
                                       double* b, double* ybuf, double* xbuf, unsigned* ctrl, bool backward,
                                       hipStream_t st, const unsigned* skip);
// fp32 variant; skip (device flag, may be null): return at once when set
hipError_t ldlt_solve_persistent(const float* K, int64_t ld, int N, const float* D, const float* P, float* b,
                                 float* ybuf, float* xbuf, unsigned* ctrl, hipStream_t st,
                                 const unsigned* skip = nullptr);

// mixed.hip: fp32 factor of S K S + fp64 iterative refinement (config C5) ----
struct MixedWs {
  int N = 0, nbo = 256;
  int64_t ld32 = 0;
  float *K32 = nullptr, *D32 = nullptr, *Linv32 = nullptr, *W32 = nullptr, *P32 = nullptr;
  float *y32 = nullptr, *z32 = nullptr, *r32 = nullptr;
  unsigned *ctrl = nullptr, *state = nullptr, *pctrl = nullptr;
  int* info = nullptr;
  double *s = nullptr, *x = nullptr, *colp = nullptr, *rowp = nullptr, *part = nullptr;
  double* stat = nullptr;  // {||r||_inf / ||b||_inf, corrections} of the last solve
  // host-mapped {done, corrections} written by the stop test, and the event
  // the host waits on before reading it (eager solves only: mixed_solve)
  unsigned *hst = nullptr, *hst_dev = nullptr;
  hipEvent_t hev = nullptr;
  int last_iters = 2;  // refinement passes the previous eager solve ran
};
int64_t mixed_ws_bytes(int N, int nbo);
int64_t mixed_ws_carve(char* base, int N, int nbo, MixedWs& w);  // base == nullptr: size only
// scale + convert + fp32 factor of the lower triangle of K (fp64, row-major)
hipError_t mixed_factor(const double* K, int64_t ld, MixedWs& w, hipStream_t st, hipStream_t st2, hipStream_t st3,
                        hipEvent_t* ev, int nev, TrailTimer* timer = nullptr, hipStream_t st4 = nullptr);
// b <- K^{-1} b by iterative refinement (device-side stop test)
hipError_t mixed_solve(const double* K, int64_t ld, MixedWs& w, double* b, double tol, int max_refine,
                       hipStream_t st);

// normal.hip: normal-equations reduction (config C2) -------------------------
hipError_t ne_check_sign(const double* D, int N, int offset, double sign, int* info, hipStream_t st);


// bk.hip: Bunch-Kaufman factor / solve (one workgroup per matrix) -----------
#define IPMZ_BK_NMAX 4096
hipError_t bk_factor(double* A, int64_t ld, int n, int* ipiv, int* info, int fix_kp, int batch, int64_t sA,
                     int64_t sP, hipStream_t st);
hipError_t bk_solve(const double* F, int64_t ld, int n, const int* ipiv, double* b, int batch, int64_t sA, int64_t sP,
                    int64_t sb, hipStream_t st);
// the whole-device factor of ONE matrix (any n; one workgroup per CU, a grid
// barrier per step): workspace bytes, launch, and its sticky error word
// (nonzero after a barrier spin timed out -- the factor is then invalid)
#define IPMZ_BK_GRID_MIN 512  // auto: the grid factor from this order up (single matrices)
size_t bk_grid_ws_bytes(int n);
hipError_t bk_factor_grid(double* A, int64_t ld, int n, int* ipiv, int* info, int fix_kp, void* ws, hipStream_t st);
const unsigned* bk_grid_err_word(const void* ws, int n);
// one system's solve through a transposed copy of the factor's lower
// triangle (LT: n x n doubles, row j = column j of L; bk_transpose once per
// factor): coalesced sweeps, the same arithmetic as bk_solve
hipError_t bk_transpose(const double* F, int64_t ld, int n, double* LT, hipStream_t st);
hipError_t bk_solve_lt(const double* LT, int n, const int* ipiv, double* b, hipStream_t st);
// Device-wide solve: A^{-1} b = P^T L'^{-T} D^{-1} L'^{-1} P b, L' = L with every
// later interchange folded into its columns (once per factor, bk_fast_prepare:
// from F, ipiv, the factor's info word and LT = bk_transpose(F); LT is
// permuted in place, L' written to the strict lower triangle of Lp, which may
// be F itself; meta: bk_fast_meta_bytes).  Then the persistent solve's
// operators are built from Lp (linv_from_l, solve_prep, solve_reset) and a
// solve is gather -> forward sweep -> dsolve (ybuf) -> backward sweep (D =
// ones) -> scatter, all gated on meta's fallback flag, + bk_fast_fallback
// (the one-workgroup sweeps on the untouched LT, run only when the flag is
// set: a singular factor, or n > 16384).
size_t bk_fast_meta_bytes(int n);
const unsigned* bk_fast_flag(const void* meta);
const double* bk_fast_ones(const void* meta, int n);
double* bk_fast_tmp(void* meta, int n);
hipError_t bk_fast_prepare(const double* F, int64_t ld, int n, const int* ipiv, const int* info, double* LT,
                           double* Lp, int64_t ldp, void* meta, hipStream_t st);
hipError_t bk_fast_gather(const double* b, int n, void* meta, hipStream_t st);
hipError_t bk_fast_dsolve(double* y, int n, void* meta, hipStream_t st);
hipError_t bk_fast_scatter(double* b, int n, void* meta, hipStream_t st);
hipError_t bk_fast_fallback(const double* LT, int n, const int* ipiv, double* b, const void* meta, hipStream_t st);

// newton.hip -----------------------------------------------------------------
enum Slot { X = 0, LA, LC, S, P, LG, LH, LY, LZ, G, H, Y, Z, NSLOT };

// device scalar block
enum Scalar {
  SC_F = 0,
  SC_RES,
  SC_MU,
  SC_ALPHA_AFF,
  SC_MU_AFF,
  SC_SIGMA,
  SC_ALPHA,
  SC_CONVERGED,
  SC_MU_NEW,
  SC_RESTARTS,
  SC_COUNT = 16
};

struct QPDev {
  int n, m, p;
  int N;
  int64_t ldn;  // leading dimension of Q, A, C (multiple of 8)
  int64_t ldk;  // leading dimension of K
  int64_t state_len;
  double delta;
  int eqnone;  // EqualityHandling::None: no p, zero (lambda_C, lambda_C) block
  int eqpen;   // EqualityHandling::PenaltyFunction: no p, -mu (lambda_C, lambda_C) block
  // Settings (oracle/ipmz_oracle.cpp QP): InequalityHandling::Slacks, and the
  // Lower / Upper halves of Settings::variable_bounds and ::inequalities
  int slacks, vlo, vup, alo, aup;
  int naive;  // InequalityHandling::NaiveSlacks: no s / lambda_A; lambda_g, lambda_h are KKT rows
  // EqualityHandling::SlackedSlacks: the p equality rows run as inequality
  // rows with l = u = d (m = m_usr + p_usr, p = 0 inside the step; the
  // formulas are the same, formulations.txt), t starting at 1
  // (EnvironmentBuilder.cpp: s_A_eq = 1).  m_usr / p_usr: the data's rows.
  int eqss, m_usr, p_usr;
  int mk;     // KKT rows of the inequalities: m, or 2 m (NaiveSlacks); N = n + mk + p
  // problem data (row-major, ld = ldn)
  const double *Q, *c, *A, *lA, *uA, *C, *d, *lx, *ux;
  double* v[NSLOT];
  double* r[NSLOT];
  double* daff[NSLOT];
  double* dir[NSLOT];
  double *Qx, *ATl, *CTl, *Ax, *Cx;
  double* b;      // augmented rhs / solution, length N
  double* scal;   // SC_COUNT doubles
  double* part;   // reduction partials
  double* tpart;  // transposed-GEMV partials: ceil(max(m, p) / IPMZ_TCHUNK) x n
  double* K;      // KKT / factor (N x ldk)
  double* K0;     // batches of small systems: the assembled KKT kept across steps (the factor reads it, writes L to K); nullptr: none
  double *v0, *r0, *scal0;  // initial iterate snapshot (benchmark restarts)
  unsigned* done;           // fused evaluation: arrival counter of the QP's workgroups (0 between launches)
};

// A batch of QPs with identical (n, m, p): d = device array of B
// descriptors (kernels index it with blockIdx.y), h = host copy of QP 0.
struct QPBatch {
  const QPDev* d;
  QPDev h;
  int B;
};

hipError_t qp_generate(const QPBatch& qb, uint64_t seed0, hipStream_t st);  // QP b: seed0 + b
hipError_t qp_init_iterate(const QPBatch& qb, hipStream_t st);
// residual vectors of the current iterate at mu = 0, plus f, res, mu,
// converged into scal (the head of Optimizer.cpp:127-135)
hipError_t qp_evaluate(const QPBatch& qb, hipStream_t st);
hipError_t qp_assemble(const QPBatch& qb, hipStream_t st);
// predictor / corrector pieces; which: 0 = affine direction, 1 = corrector
hipError_t qp_rhs(const QPBatch& qb, hipStream_t st);
hipError_t qp_backsub(const QPBatch& qb, int which, hipStream_t st);
hipError_t qp_ratio(const QPBatch& qb, int which, int out_index, hipStream_t st);
hipError_t qp_mu_aff(const QPBatch& qb, hipStream_t st);
hipError_t qp_corrector_residuals(const QPBatch& qb, hipStream_t st);
hipError_t qp_update(const QPBatch& qb, int freeze, hipStream_t st);
hipError_t qp_restart_if_converged(const QPBatch& qb, hipStream_t st);
hipError_t qp_save_initial(const QPBatch& qb, hipStream_t st);
// out (device, 3 doubles) = {max res, max mu, unconverged count} over the batch
hipError_t qp_batch_summary(const QPBatch& qb, double* out, hipStream_t st);
// Fused per-QP phases for batches of small systems (one workgroup per QP):
// pre = restart-if-converged + assembly + affine rhs (+ info word reset),
// mid = predictor back-substitution .. corrector rhs, post = corrector
// back-substitution + update + evaluation.  N <= IPMZ_FUSED_NMAX.
#define IPMZ_FUSED_NMAX 1024
// kmode: 0 = the whole lower triangle into K; 1 = the diagonal into K0 (its
// off-diagonal part is already there); 2 = only the off-diagonal part into
// K0 (once per data load; no restart, no rhs)
enum { KMODE_K = 0, KMODE_K0_DIAG = 1, KMODE_K0_OFFDIAG = 2 };
hipError_t qp_fused_pre(const QPBatch& qb, int restart, int* info, hipStream_t st, int kmode = KMODE_K);
hipError_t qp_fused_mid(const QPBatch& qb, hipStream_t st);
hipError_t qp_fused_post(const QPBatch& qb, int freeze, hipStream_t st);  // (+ the evaluation)
// predictor solve + mid + corrector solve + post in one workgroup per QP
// (the small batched solve, ldlt_solve_batched's nbi = 64 path: N <=
// TRSV_SMALL_NMAX, even ld), then the evaluation alone
inline bool fused_solves_ok(int N, int64_t ld) { return N <= 4096 && !(ld & 1); }
hipError_t qp_fused_solves(const QPBatch& qb, const double* K, int64_t ld, int N, const double* D, const double* Linv,
                           double* b, int64_t sK, int64_t sD, int64_t sL, int64_t sb, int freeze, hipStream_t st);
hipError_t qp_fused_eval(const QPBatch& qb, hipStream_t st);

}  // namespace ipmz
