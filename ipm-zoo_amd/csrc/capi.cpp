// C ABI of libipmz (include/ipmz.h): contexts, the LinearSolvers entry
// points and the Newton-step solver object.  Host orchestration only -- all
// arithmetic runs in the gfx950 kernels of ldlt.hip / trsv.hip / newton.hip.
// There is deliberately no CPU fallback: without a device every computing
// entry point fails with IPMZ_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "ipmz.h"
#include "kernels.h"

using namespace ipmz;

namespace {
thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
#define HIP_OK(expr)                                                                                     \
  do {                                                                                                   \
    hipError_t _e = (expr);                                                                              \
    if (_e != hipSuccess)                                                                                \
      return fail(IPMZ_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e) + " @" + __FILE__ + ":" + \
                                    std::to_string(__LINE__));                                           \
  } while (0)

int64_t round_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }
int ws_status(hipStream_t st, const char* ws, int N, int nbo, int nbi, const char* what);
int err_words_status(hipStream_t st, const unsigned* pe, const unsigned* se, const char* what);

}  // namespace

struct ipmz_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  int nbo = 0, nbi = 64;  // nbo 0: by matrix order (nbo_for)
  // factorization look-ahead: the panel chain on `stream` itself, panel rows
  // on sC (high priority), trailing updates on sB, the fp32 factor's
  // look-ahead strips on sD; forked from / joined to `stream` (ldlt_factor)
  hipStream_t sB = nullptr, sC = nullptr, sD = nullptr;
  std::vector<hipEvent_t> evpool;
  // the sticky error words (spin timeouts of the persistent kernels) of the
  // workspace the last asynchronous device-memory solve used, resolved when
  // it was enqueued: ipmz_ctx_sync checks and clears them (the caller keeps
  // that workspace alive until then)
  const unsigned* check_pe = nullptr;
  const unsigned* check_se = nullptr;
  // solvers created on this context and not yet destroyed: a context
  // destroyed before them (e.g. a garbage collector finalizing both in either
  // order) is only marked, and freed with the last of them.  Both fields are
  // read and written only under g_ctx_mutex (ctypes drops the GIL around
  // every call, and finalizers run on any thread).
  int users = 0;
  bool closed = false;
};

static std::mutex g_ctx_mutex;

// outer panel width for an order-N factor: the context's, or by size --
// 512 for N > 4096 (kbench factor, N = 11264: 12.95 ms at 384, 12.34 at
// 512; N = 16384: 32.1 -> 31.2 ms), 384 for 2048 <= N <= 4096 (C2, N = 2560,
// chain-bound: 679-689 steps/s at 512, 711-718 at 384 in round 5,
// profiles/r05_s/c2_nbo_ab.txt; 256: 675), 256 below.  Every workspace
// layout and every factor / solve of an order-N matrix uses this same value.
static int nbo_for(const ipmz_ctx* ctx, int N) {
  if (ctx->nbo > 0) return ctx->nbo;
  if (ctx->nbi != 64 || N < 2048) return 256;
  return N <= 4096 ? 384 : 512;
}

// The pool's events only order the factor's streams on one device: no
// system-scope release / acquire fence when one is recorded or waited for
// (the default writes the L2 back for the host at every record, on the
// panel chain's stream between every two chain launches); a runtime that
// refuses the flag gets the default events
static int ensure_events(ipmz_ctx* ctx, size_t n) {
  while (ctx->evpool.size() < n) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess &&
        hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
      return fail(IPMZ_ERR_HIP, "hipEventCreate failed");
    ctx->evpool.push_back(e);
  }
  return IPMZ_OK;
}

// the end of a factorization that forked onto the look-ahead streams: the
// caller's stream waits for each of them (the chain stream A has already
// waited for B's and C's work; the explicit waits keep every stream a capture
// forked joined back into its origin -- ldlt.hip stream_wait)
static int check_device(int device) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
    return fail(IPMZ_ERR_NO_DEVICE, "no HIP device visible: libipmz has no CPU fallback");
  if (device < 0 || device >= count) return fail(IPMZ_ERR_INVALID, "device index out of range");
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return fail(IPMZ_ERR_NO_DEVICE, "device query failed");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(IPMZ_ERR_NO_DEVICE, std::string("libipmz is built for gfx950, device is ") + prop.gcnArchName);
  return IPMZ_OK;
}

extern "C" {

const char* ipmz_last_error(void) { return g_last_error.c_str(); }

int ipmz_ctx_create(ipmz_ctx** out, int device) {
  if (!out) return fail(IPMZ_ERR_INVALID, "null out");
  *out = nullptr;
  int rc = check_device(device);
  if (rc) return rc;
  HIP_OK(hipSetDevice(device));
  auto* c = new ipmz_ctx();
  c->device = device;
  int least = 0, greatest = 0;
  hipDeviceGetStreamPriorityRange(&least, &greatest);
  // own: the steps' stream, and the factor's panel chain (high priority)
  if (hipStreamCreateWithPriority(&c->own, hipStreamNonBlocking, greatest) != hipSuccess) {
    delete c;
    return fail(IPMZ_ERR_HIP, "hipStreamCreate failed");
  }
  c->stream = c->own;
  if (hipStreamCreateWithPriority(&c->sB, hipStreamNonBlocking, least) != hipSuccess ||
      hipStreamCreateWithPriority(&c->sC, hipStreamNonBlocking, greatest) != hipSuccess ||
      hipStreamCreateWithPriority(&c->sD, hipStreamNonBlocking, greatest) != hipSuccess) {
    ipmz_ctx_destroy(c);
    return fail(IPMZ_ERR_HIP, "hipStreamCreateWithPriority failed");
  }
  *out = c;
  return IPMZ_OK;
}

static void ctx_free(ipmz_ctx* ctx) {
  hipSetDevice(ctx->device);
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  for (hipStream_t s : {ctx->own, ctx->sB, ctx->sC, ctx->sD})
    if (s) {
      hipStreamSynchronize(s);
      hipStreamDestroy(s);
    }
  for (auto e : ctx->evpool) hipEventDestroy(e);
  delete ctx;
}

int ipmz_ctx_destroy(ipmz_ctx* ctx) {
  if (!ctx) return IPMZ_OK;
  {
    std::lock_guard<std::mutex> lk(g_ctx_mutex);
    if (ctx->closed) return IPMZ_OK;
    ctx->closed = true;
    if (ctx->users > 0) {
      // freed with its last solver: from now on the solvers run on the
      // context's own stream, so that late free never touches a caller's
      // stream whose owner may have released it after this call (what the
      // solvers enqueued there is drained first)
      if (ctx->stream != ctx->own) {
        hipSetDevice(ctx->device);
        hipStreamSynchronize(ctx->stream);
      }
      ctx->stream = ctx->own;
      return IPMZ_OK;
    }
  }
  ctx_free(ctx);
  return IPMZ_OK;
}

int ipmz_ctx_set_stream(ipmz_ctx* ctx, void* s) {
  if (!ctx) return fail(IPMZ_ERR_INVALID, "null ctx");
  ctx->stream = static_cast<hipStream_t>(s);  // NULL = the legacy default stream
  return IPMZ_OK;
}

int ipmz_ctx_reset_stream(ipmz_ctx* ctx) {
  if (!ctx) return fail(IPMZ_ERR_INVALID, "null ctx");
  ctx->stream = ctx->own;
  return IPMZ_OK;
}

int ipmz_ctx_sync(ipmz_ctx* ctx) {
  if (!ctx) return fail(IPMZ_ERR_INVALID, "null ctx");
  HIP_OK(hipStreamSynchronize(ctx->stream));
  if (ctx->check_pe) {
    const unsigned *pe = ctx->check_pe, *se = ctx->check_se;
    ctx->check_pe = ctx->check_se = nullptr;
    return err_words_status(ctx->stream, pe, se, "ipmz_ctx_sync");
  }
  return IPMZ_OK;
}

int ipmz_debug_inject(int mask) {
  set_debug_inject_mask(mask);
  return IPMZ_OK;
}

int ipmz_ctx_set_blocking(ipmz_ctx* ctx, int nbo, int nbi) {
  if (!ctx) return fail(IPMZ_ERR_INVALID, "null ctx");
  if ((nbi != 64 && nbi != 128) || (nbo != 0 && (nbo < nbi || nbo % nbi != 0 || nbo > IPMZ_NBO_MAX)))
    return fail(IPMZ_ERR_INVALID, "blocking: nbi in {64,128}, nbo 0 (auto) or a multiple of nbi, <= 512");
  ctx->nbo = nbo;
  ctx->nbi = nbi;
  return IPMZ_OK;
}

int ipmz_ctx_get_blocking(ipmz_ctx* ctx, int N, int* nbo, int* nbi) {
  if (!ctx || N < 0 || !nbo || !nbi) return fail(IPMZ_ERR_INVALID, "ipmz_ctx_get_blocking: bad arguments");
  *nbo = nbo_for(ctx, N);
  *nbi = ctx->nbi;
  return IPMZ_OK;
}

// ---------------------------------------------------------------------------
// Workspace: [info int (256 B)] [panel ctrl words] [side 2*nbi] [Linv nblk*nbi^2] [W 3*N*nbo]
//            [ybuf N] [zbuf N] [solve ctrl words] [solve prep (nbi 64): X, X^T, M, Q per 128-row block]
namespace {
struct WsLayout {
  int64_t info_off, pctrl_off, side_off, linv_off, w_off, y_off, z_off, ctrl_off, prep_off, total;
};
WsLayout ws_layout(int N, int nbo, int nbi) {
  WsLayout l;
  const int64_t nblk = (N + nbi - 1) / nbi;
  l.info_off = 0;
  l.pctrl_off = 256;  // panel_ctrl_words(N, nbo) words
  l.side_off = l.pctrl_off + round_up(panel_ctrl_words(N, nbo) * 4, 256);
  l.linv_off = l.side_off + round_up(2 * nbi * 8, 256);
  l.w_off = l.linv_off + round_up(nblk * nbi * nbi * 8, 256);
  l.y_off = l.w_off + round_up(3 * (int64_t)N * nbo * 8, 256);  // W triple-buffered (look-ahead)
  l.z_off = l.y_off + round_up((int64_t)N * 8, 256);
  l.ctrl_off = l.z_off + round_up((int64_t)N * 8, 256);
  l.prep_off = l.ctrl_off + 256;
  l.total = l.prep_off + (nbi == 64 ? round_up(solve_prep_elems(N) * 8, 256) : 0);
  return l;
}
// the solve: one persistent launch for nbi == 64 (trsv_persist.hip), else
// the block-step kernel chain (trsv.hip)
hipError_t solve_ws(const double* K, int64_t ld, int N, const double* D, const char* ws, int nbo, int nbi, double* b,
                    hipStream_t st) {
  const WsLayout l = ws_layout(N, nbo, nbi);
  char* w = const_cast<char*>(ws);
  const double* Linv = reinterpret_cast<const double*>(w + l.linv_off);
  if (nbi == 64)
    return ldlt_solve_persistent(K, ld, N, D, reinterpret_cast<const double*>(w + l.prep_off), b,
                                 reinterpret_cast<double*>(w + l.y_off), reinterpret_cast<double*>(w + l.z_off),
                                 reinterpret_cast<unsigned*>(w + l.ctrl_off), st);
  return ldlt_solve(K, ld, N, D, Linv, nbi, b, reinterpret_cast<double*>(w + l.side_off), st);
}
// Sticky error words of a workspace (synchronizes): a spin that timed out in
// the outer-panel factor or the persistent solve (sync.h, 0.5 s) means the
// results are invalid -- reported as IPMZ_ERR_HIP, never as success.
const unsigned* panel_err_word(const char* ws, const WsLayout& l) {
  return reinterpret_cast<const unsigned*>(ws + l.pctrl_off) + PANEL_ERR_WORD;
}
const unsigned* solve_err_word(const char* ws, const WsLayout& l) {
  return reinterpret_cast<const unsigned*>(ws + l.ctrl_off) + SOLVE_ERR_WORD;
}
int ws_status(hipStream_t st, const char* ws, int N, int nbo, int nbi, const char* what) {
  const WsLayout l = ws_layout(N, nbo, nbi);
  return err_words_status(st, panel_err_word(ws, l), solve_err_word(ws, l), what);
}
int err_words_status(hipStream_t st, const unsigned* pe_word, const unsigned* se_word, const char* what) {
  unsigned pe = 0, se = 0;
  HIP_OK(hipMemcpyAsync(&pe, pe_word, 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(&se, se_word, 4, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  if (pe) return fail(IPMZ_ERR_HIP, std::string(what) + ": a hand-off inside the outer-panel factor kernel timed out "
                                                        "(spin limit 0.5 s); the factor is invalid");
  if (se) return fail(IPMZ_ERR_HIP, std::string(what) + ": a hand-off inside the persistent triangular solve timed out "
                                                        "(spin limit 0.5 s); the solution is invalid");
  return IPMZ_OK;
}
}  // namespace

}  // extern "C"

// The device-wide Bunch-Kaufman solve's workspace (bk.hip bk_fast_*): the
// persistent triangular solve's operators for L' (64 x 64 inverse diagonal
// blocks, the 128-row-block prep), its y / x vectors and ctrl words, and the
// interchange bookkeeping (meta)
namespace {
struct BkWs {
  double *Linv = nullptr, *P = nullptr, *y = nullptr, *x = nullptr;
  unsigned* ctrl = nullptr;
  char* meta = nullptr;
  int64_t total = 0;
};
BkWs bk_ws(char* base, int N) {
  BkWs w;
  int64_t off = 0;
  auto take = [&](int64_t bytes) {
    char* p = base ? base + off : nullptr;
    off += round_up(bytes, 256);
    return p;
  };
  w.Linv = reinterpret_cast<double*>(take((int64_t)((N + 63) / 64) * 64 * 64 * 8));
  w.P = reinterpret_cast<double*>(take(solve_prep_elems(N) * 8));
  w.y = reinterpret_cast<double*>(take((int64_t)N * 8));
  w.x = reinterpret_cast<double*>(take((int64_t)N * 8));
  w.ctrl = reinterpret_cast<unsigned*>(take(256));
  w.meta = take((int64_t)bk_fast_meta_bytes(N));
  w.total = off;
  return w;
}
// once per factor: L' (into Lp, may be F), then the persistent solve's operators
hipError_t bk_setup(const double* F, int64_t ld, int N, const int* ipiv, const int* info, double* LT, double* Lp,
                    int64_t ldp, const BkWs& w, hipStream_t st) {
  hipError_t e = bk_fast_prepare(F, ld, N, ipiv, info, LT, Lp, ldp, w.meta, st);
  if (e == hipSuccess) e = linv_from_l(Lp, ldp, N, 64, w.Linv, st);
  if (e == hipSuccess) e = solve_prep(Lp, ldp, N, w.Linv, w.P, st);
  if (e == hipSuccess) e = solve_reset(w.y, w.x, sizeof(double), N, w.ctrl, st);
  return e;
}
// b <- A^{-1} b: P^T L'^{-T} D^{-1} L'^{-1} P b, or the one-workgroup sweeps on
// LT when the factor needs the reference's exact interchange order
hipError_t bk_run(const double* Lp, int64_t ldp, int N, const double* LT, const int* ipiv, const BkWs& w, double* b,
                  hipStream_t st) {
  const unsigned* flag = bk_fast_flag(w.meta);
  double* t = bk_fast_tmp(w.meta, N);
  const double* ones = bk_fast_ones(w.meta, N);
  hipError_t e = bk_fast_gather(b, N, w.meta, st);
  if (e == hipSuccess) e = ldlt_solve_persistent_sweep(Lp, ldp, N, ones, w.P, t, w.y, w.x, w.ctrl, false, st, flag);
  if (e == hipSuccess) e = bk_fast_dsolve(w.y, N, w.meta, st);
  if (e == hipSuccess) e = ldlt_solve_persistent_sweep(Lp, ldp, N, ones, w.P, t, w.y, w.x, w.ctrl, true, st, flag);
  if (e == hipSuccess) e = bk_fast_scatter(b, N, w.meta, st);
  if (e == hipSuccess) e = bk_fast_fallback(LT, N, ipiv, b, w.meta, st);
  return e;
}
}  // namespace

extern "C" {

int64_t ipmz_ldlt_workspace_bytes(ipmz_ctx* ctx, int N) {
  if (!ctx || N < 0) return 0;
  return ws_layout(N, nbo_for(ctx, N), ctx->nbi).total;
}

// info2: a caller's own info word, reset in the same launch
static int factor_impl(ipmz_ctx* ctx, int N, double* K, int64_t ld, double* D, char* ws, TrailTimer* timer,
                       int* info2 = nullptr) {
  const WsLayout l = ws_layout(N, nbo_for(ctx, N), ctx->nbi);
  int* info = reinterpret_cast<int*>(ws + l.info_off);
  double* Linv = reinterpret_cast<double*>(ws + l.linv_off);
  double* W = reinterpret_cast<double*>(ws + l.w_off);
  unsigned* pctrl = reinterpret_cast<unsigned*>(ws + l.pctrl_off);
  // one launch: info, the panel ctrl words and the persistent solve's state
  // for this factor
  HIP_OK(solve_reset(ws + l.y_off, ws + l.z_off, sizeof(double), N, reinterpret_cast<unsigned*>(ws + l.ctrl_off),
                     ctx->stream, info, pctrl, panel_ctrl_words(N, nbo_for(ctx, N)), info2));
  const int nbo = nbo_for(ctx, N);
  const int npan = (N + nbo - 1) / nbo;
  // the persistent solve's per-block operators, built once from this factor
  auto prep = [&]() -> hipError_t {
    return ctx->nbi == 64 ? solve_prep(K, ld, N, Linv, reinterpret_cast<double*>(ws + l.prep_off), ctx->stream)
                          : hipSuccess;
  };
  if (npan < 3 || (debug_inject_mask() & IPMZ_DEBUG_ONE_STREAM)) {
    HIP_OK(ldlt_factor(K, ld, N, D, Linv, W, nbo, ctx->nbi, info, ctx->stream, timer, nullptr, nullptr, nullptr, 0,
                       pctrl));
    HIP_OK(prep());
    return IPMZ_OK;
  }
  const int nev = 5 * npan + 5;  // ldlt_factor's 5 npan + 3, the fork, one spare
  int rc = ensure_events(ctx, (size_t)nev + 4);
  if (rc) return rc;
  hipEvent_t* ev = ctx->evpool.data();
  // the fourth look-ahead stream pays for the fp32 factor only (C5 23.6 ->
  // 22.9 ms per step); the fp64 one runs faster without it (C3 14.2 -> 14.0
  // ms), profiles/r03_s5/fourth_stream_ab.log -- not forked at all here
  const bool fourth = false;
  // the panel chain on the caller's stream itself: its first launch follows
  // the assembly in stream order, with no cross-queue hop; ldlt_factor forks
  // B (trailing updates) and C (rows launches) from it and joins them back
  // (a fork onto A cost the C2 step ~70 us of host enqueue before the first
  // panel, profiles/r05_s18)
  HIP_OK(ldlt_factor(K, ld, N, D, Linv, W, nbo, ctx->nbi, info, ctx->stream, timer, ctx->sB, ctx->sC, ev, nev - 2,
                     pctrl, fourth ? ctx->sD : nullptr));
  HIP_OK(prep());
  return IPMZ_OK;
}

// info word (first non-finite pivot) + the sticky error words of ws
static int read_info(ipmz_ctx* ctx, const char* ws, int N) {
  int rc = ws_status(ctx->stream, ws, N, nbo_for(ctx, N), ctx->nbi, "ipmz_ldlt_factor");
  if (rc) return rc;
  int info = 0;
  HIP_OK(hipMemcpyAsync(&info, ws, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  return info == 0x7f7f7f7f ? IPMZ_OK : info;
}

int ipmz_ldlt_factor(ipmz_ctx* ctx, int N, double* K, int64_t ld, double* D, void* ws, int64_t ws_bytes) {
  if (!ctx || N < 0 || (N > 0 && (!K || !D || !ws)) || ld < N || (ld & 1))
    return fail(IPMZ_ERR_INVALID, "ipmz_ldlt_factor: bad arguments (ld >= N, ld even)");
  if (N == 0) return IPMZ_OK;
  if (ws_bytes < ws_layout(N, nbo_for(ctx, N), ctx->nbi).total) return fail(IPMZ_ERR_INVALID, "workspace too small");
  HIP_OK(hipSetDevice(ctx->device));
  int rc = factor_impl(ctx, N, K, ld, D, static_cast<char*>(ws), nullptr);
  if (rc) return rc;
  return read_info(ctx, static_cast<char*>(ws), N);  // synchronous: checks the error words itself
}

int ipmz_ldlt_solve(ipmz_ctx* ctx, int N, const double* K, int64_t ld, const double* D, const void* ws, double* b) {
  if (!ctx || N < 0 || ld < N) return fail(IPMZ_ERR_INVALID, "ipmz_ldlt_solve: bad arguments");
  if (N == 0) return IPMZ_OK;
  HIP_OK(hipSetDevice(ctx->device));
  HIP_OK(solve_ws(K, ld, N, D, static_cast<const char*>(ws), nbo_for(ctx, N), ctx->nbi, b, ctx->stream));
  // its error words are checked by ipmz_ctx_sync (addresses resolved now: a
  // later ipmz_ctx_set_blocking does not move them)
  const WsLayout l = ws_layout(N, nbo_for(ctx, N), ctx->nbi);
  ctx->check_pe = panel_err_word(static_cast<const char*>(ws), l);
  ctx->check_se = solve_err_word(static_cast<const char*>(ws), l);
  return IPMZ_OK;
}

int ipmz_ldlt_prepare_solve(ipmz_ctx* ctx, int N, const double* L, int64_t ld, void* ws, int64_t ws_bytes) {
  if (!ctx || N < 0 || ld < N) return fail(IPMZ_ERR_INVALID, "ipmz_ldlt_prepare_solve: bad arguments");
  if (N == 0) return IPMZ_OK;
  if (ws_bytes < ws_layout(N, nbo_for(ctx, N), ctx->nbi).total) return fail(IPMZ_ERR_INVALID, "workspace too small");
  HIP_OK(hipSetDevice(ctx->device));
  const WsLayout l = ws_layout(N, nbo_for(ctx, N), ctx->nbi);
  HIP_OK(linv_from_l(L, ld, N, ctx->nbi, reinterpret_cast<double*>(static_cast<char*>(ws) + l.linv_off),
                     ctx->stream));
  if (ctx->nbi == 64)
    HIP_OK(solve_prep(L, ld, N, reinterpret_cast<const double*>(static_cast<char*>(ws) + l.linv_off),
                      reinterpret_cast<double*>(static_cast<char*>(ws) + l.prep_off), ctx->stream));
  // no factorization ran in this workspace: clear its sticky error words
  HIP_OK(solve_reset(static_cast<char*>(ws) + l.y_off, static_cast<char*>(ws) + l.z_off, sizeof(double), N,
                     reinterpret_cast<unsigned*>(static_cast<char*>(ws) + l.ctrl_off), ctx->stream, nullptr,
                     reinterpret_cast<unsigned*>(static_cast<char*>(ws) + l.pctrl_off),
                     panel_ctrl_words(N, nbo_for(ctx, N))));
  return IPMZ_OK;
}

// Mixed precision (config C5) -------------------------------------------------
}  // extern "C"

// factor of S K S in fp32, with the same two-stream look-ahead as the fp64 factor
static int mixed_factor_impl(ipmz_ctx* ctx, const double* K, int64_t ld, MixedWs& w, TrailTimer* timer) {
  const int npan = (w.N + w.nbo - 1) / w.nbo;
  if (npan < 3 || (debug_inject_mask() & IPMZ_DEBUG_ONE_STREAM)) {
    HIP_OK(mixed_factor(K, ld, w, ctx->stream, nullptr, nullptr, nullptr, 0, timer));
    HIP_OK(solve_prep(w.K32, w.ld32, w.N, w.Linv32, w.P32, ctx->stream));
    return IPMZ_OK;
  }
  const int nev = 5 * npan + 5;  // ldlt_factor's 5 npan + 3, the fork, one spare
  int rc = ensure_events(ctx, (size_t)nev + 4);
  if (rc) return rc;
  hipEvent_t* ev = ctx->evpool.data();
  const bool fourth = !(debug_inject_mask() & IPMZ_DEBUG_NO_FOURTH);
  // the chain on the caller's stream (factor_impl); ldlt_factor forks and
  // joins B, C and D
  HIP_OK(mixed_factor(K, ld, w, ctx->stream, ctx->sB, ctx->sC, ev, nev - 2, timer, fourth ? ctx->sD : nullptr));
  HIP_OK(solve_prep(w.K32, w.ld32, w.N, w.Linv32, w.P32, ctx->stream));
  return IPMZ_OK;
}

extern "C" {

int64_t ipmz_mixed_workspace_bytes(ipmz_ctx* ctx, int N) {
  if (!ctx || N < 0) return 0;
  return mixed_ws_bytes(N, nbo_for(ctx, N));
}

int ipmz_mixed_factor(ipmz_ctx* ctx, int N, const double* K, int64_t ld, void* ws, int64_t ws_bytes) {
  if (!ctx || N < 0 || (N > 0 && (!K || !ws)) || ld < N) return fail(IPMZ_ERR_INVALID, "ipmz_mixed_factor: bad arguments");
  if (N == 0) return IPMZ_OK;
  if (ws_bytes < mixed_ws_bytes(N, nbo_for(ctx, N))) return fail(IPMZ_ERR_INVALID, "workspace too small");
  HIP_OK(hipSetDevice(ctx->device));
  MixedWs w;
  mixed_ws_carve(static_cast<char*>(ws), N, nbo_for(ctx, N), w);
  int rc = mixed_factor_impl(ctx, K, ld, w, nullptr);
  if (rc) return rc;
  int info = 0;
  HIP_OK(hipMemcpyAsync(&info, w.info, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  return info == 0x7f7f7f7f ? IPMZ_OK : info;
}

int ipmz_mixed_solve(ipmz_ctx* ctx, int N, const double* K, int64_t ld, void* ws, double* b, double tol,
                     int max_refine, double* stat) {
  if (!ctx || N < 0 || ld < N || max_refine < 0) return fail(IPMZ_ERR_INVALID, "ipmz_mixed_solve: bad arguments");
  if (N == 0) return IPMZ_OK;
  if (!K || !ws || !b) return fail(IPMZ_ERR_INVALID, "null pointer");
  HIP_OK(hipSetDevice(ctx->device));
  MixedWs w;
  mixed_ws_carve(static_cast<char*>(ws), N, nbo_for(ctx, N), w);
  HIP_OK(mixed_solve(K, ld, w, b, tol, max_refine, ctx->stream));
  if (stat) {
    HIP_OK(hipMemcpyAsync(stat, w.stat, 2 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIP_OK(hipStreamSynchronize(ctx->stream));
  }
  return IPMZ_OK;
}

// Normal equations (config C2) ---------------------------------------------
}  // extern "C"

namespace {
// [definiteness info (256 B)] [ws of the order n + mp LDL^T]
struct NormalWs {
  int* info = nullptr;
  char* wsK = nullptr;
  int64_t total = 0;
};
NormalWs normal_ws(char* base, int n, int mp, const ipmz_ctx* ctx) {
  NormalWs w;
  w.info = reinterpret_cast<int*>(base);
  w.wsK = base ? base + 256 : nullptr;
  w.total = 256 + ws_layout(n + mp, nbo_for(ctx, n + mp), ctx->nbi).total;
  return w;
}
}  // namespace

// The normal equations as the x-first blocked LDL^T of [[H, B^T], [B, -E]]
// (normal.hip): Cholesky(H), the TRSM of B, the SYRK into the (2,2) block and
// Cholesky(S) in one pipelined factor; then H's pivots > 0, S's < 0.
static int normal_factor_impl(ipmz_ctx* ctx, int n, int mp, double* K, int64_t ld, double* D, const NormalWs& w,
                              TrailTimer* timer) {
  hipStream_t st = ctx->stream;
  int rc = factor_impl(ctx, n + mp, K, ld, D, w.wsK, timer, w.info);
  if (rc) return rc;
  HIP_OK(ne_check_sign(D, n, 0, 1.0, w.info, st));
  HIP_OK(ne_check_sign(D + n, mp, n, -1.0, w.info, st));
  return IPMZ_OK;
}

// b = [r0; r1] <- [x; l]: the factor's forward and backward sweeps
static int normal_solve_impl(ipmz_ctx* ctx, int n, int mp, const double* K, int64_t ld, const double* D,
                             const NormalWs& w, double* b) {
  HIP_OK(solve_ws(K, ld, n + mp, D, w.wsK, nbo_for(ctx, n + mp), ctx->nbi, b, ctx->stream));
  return IPMZ_OK;
}

extern "C" {

int64_t ipmz_normal_workspace_bytes(ipmz_ctx* ctx, int n, int mp) {
  if (!ctx || n <= 0 || mp < 0) return 0;
  return normal_ws(nullptr, n, mp, ctx).total;
}

int ipmz_normal_factor(ipmz_ctx* ctx, int n, int mp, double* K, int64_t ld, double* D, void* ws, int64_t ws_bytes) {
  if (!ctx || n <= 0 || mp < 0 || !K || !D || !ws || ld < n + mp || (ld & 1))
    return fail(IPMZ_ERR_INVALID, "ipmz_normal_factor: bad arguments (n > 0, ld >= n + mp, ld even)");
  const NormalWs w = normal_ws(static_cast<char*>(ws), n, mp, ctx);
  if (ws_bytes < w.total) return fail(IPMZ_ERR_INVALID, "workspace too small");
  HIP_OK(hipSetDevice(ctx->device));
  int rc = normal_factor_impl(ctx, n, mp, K, ld, D, w, nullptr);
  if (rc) return rc;
  int info = 0;
  HIP_OK(hipMemcpyAsync(&info, w.info, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  if (info != 0x7f7f7f7f) return info;
  return read_info(ctx, w.wsK, n + mp);  // a non-finite pivot of the factor
}

int ipmz_normal_solve(ipmz_ctx* ctx, int n, int mp, const double* K, int64_t ld, const double* D, void* ws,
                      double* b) {
  if (!ctx || n <= 0 || mp < 0 || !K || !D || !ws || !b || ld < n + mp)
    return fail(IPMZ_ERR_INVALID, "ipmz_normal_solve: bad arguments");
  HIP_OK(hipSetDevice(ctx->device));
  return normal_solve_impl(ctx, n, mp, K, ld, D, normal_ws(static_cast<char*>(ws), n, mp, ctx), b);
}

// Bunch-Kaufman (f3) ----------------------------------------------------------
int ipmz_bk_factor(ipmz_ctx* ctx, int N, double* A, int64_t ld, int* ipiv, int fix_kp) {
  return ipmz_bk_factor_ex(ctx, N, A, ld, ipiv, fix_kp, IPMZ_BK_AUTO);
}

int ipmz_bk_factor_ex(ipmz_ctx* ctx, int N, double* A, int64_t ld, int* ipiv, int fix_kp, int algo) {
  if (!ctx || N < 0 || ld < N || (N > 0 && (!A || !ipiv)) || algo < IPMZ_BK_AUTO || algo > IPMZ_BK_GRID)
    return fail(IPMZ_ERR_INVALID, "ipmz_bk_factor: bad arguments");
  const bool grid = algo == IPMZ_BK_GRID || (algo == IPMZ_BK_AUTO && N >= IPMZ_BK_GRID_MIN);
  if (!grid && N > IPMZ_BK_NMAX) return fail(IPMZ_ERR_INVALID, "ipmz_bk_factor: N > 4096 for the one-workgroup factor");
  if (N == 0) return IPMZ_OK;
  HIP_OK(hipSetDevice(ctx->device));
  const size_t wsb = grid ? bk_grid_ws_bytes(N) : 0;
  char* dws = nullptr;
  HIP_OK(hipMallocAsync(reinterpret_cast<void**>(&dws), 256 + wsb, ctx->stream));
  int* dinfo = reinterpret_cast<int*>(dws);
  int rc = IPMZ_OK, info = 0;
  unsigned err = 0;
  const hipError_t e = grid ? bk_factor_grid(A, ld, N, ipiv, dinfo, fix_kp, dws + 256, ctx->stream)
                            : bk_factor(A, ld, N, ipiv, dinfo, fix_kp, 1, 0, 0, ctx->stream);
  if (e != hipSuccess || hipMemcpyAsync(&info, dinfo, sizeof(int), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
      (grid && hipMemcpyAsync(&err, bk_grid_err_word(dws + 256, N), 4, hipMemcpyDeviceToHost, ctx->stream) !=
                   hipSuccess) ||
      hipStreamSynchronize(ctx->stream) != hipSuccess)
    rc = fail(IPMZ_ERR_HIP, "ipmz_bk_factor: launch failed");
  else if (err)
    rc = fail(IPMZ_ERR_HIP, "ipmz_bk_factor: a grid barrier of the whole-device factor timed out; the factor is invalid");
  hipFreeAsync(dws, ctx->stream);
  return rc ? rc : info;
}

int ipmz_bk_solve(ipmz_ctx* ctx, int N, const double* F, int64_t ld, const int* ipiv, double* b) {
  if (!ctx || N < 0 || ld < N) return fail(IPMZ_ERR_INVALID, "ipmz_bk_solve: bad arguments");
  if (N == 0) return IPMZ_OK;  // LinearSolvers.cpp:212-214
  if (!F || !ipiv || !b) return fail(IPMZ_ERR_INVALID, "null pointer");
  HIP_OK(hipSetDevice(ctx->device));
  if (N < IPMZ_BK_GRID_MIN) {
    HIP_OK(bk_solve(F, ld, N, ipiv, b, 1, 0, 0, 0, ctx->stream));
    return IPMZ_OK;
  }
  // large N: the device-wide solve (L' with the interchanges folded in,
  // built here from F into stream-ordered buffers, freed after the solve)
  const int64_t ldp = round_up(N, 64);
  const BkWs wsz = bk_ws(nullptr, N);
  double *lt = nullptr, *lp = nullptr;
  char* wb = nullptr;
  HIP_OK(hipMallocAsync(reinterpret_cast<void**>(&lt), (size_t)N * N * sizeof(double), ctx->stream));
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&lp), (size_t)N * ldp * sizeof(double), ctx->stream);
  if (e == hipSuccess) e = hipMallocAsync(reinterpret_cast<void**>(&wb), (size_t)wsz.total, ctx->stream);
  const BkWs w = bk_ws(wb, N);
  if (e == hipSuccess) e = bk_transpose(F, ld, N, lt, ctx->stream);
  if (e == hipSuccess) e = bk_setup(F, ld, N, ipiv, nullptr, lt, lp, ldp, w, ctx->stream);
  if (e == hipSuccess) e = bk_run(lp, ldp, N, lt, ipiv, w, b, ctx->stream);
  unsigned serr = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&serr, w.ctrl + SOLVE_ERR_WORD, 4, hipMemcpyDeviceToHost, ctx->stream);
  if (wb) hipFreeAsync(wb, ctx->stream);
  if (lp) hipFreeAsync(lp, ctx->stream);
  hipFreeAsync(lt, ctx->stream);
  HIP_OK(e);
  HIP_OK(hipStreamSynchronize(ctx->stream));
  if (serr) return fail(IPMZ_ERR_HIP, "ipmz_bk_solve: a hand-off inside the persistent triangular solve timed out "
                                      "(spin limit 0.5 s); the solution is invalid");
  return IPMZ_OK;
}

int ipmz_symmetric_indefinite_factorization(ipmz_ctx* ctx, int N, const double* A, double* F, int* ipiv) {
  if (!ctx || N < 0 || (N > 0 && (!A || !F || !ipiv)))
    return fail(IPMZ_ERR_INVALID, "ipmz_symmetric_indefinite_factorization: bad arguments");
  if (N == 0) return IPMZ_OK;
  HIP_OK(hipSetDevice(ctx->device));
  double* dA = nullptr;
  int* dp = nullptr;
  if (hipMalloc(&dA, (size_t)N * N * 8) != hipSuccess || hipMalloc(&dp, (size_t)N * 4) != hipSuccess) {
    hipFree(dA);
    return fail(IPMZ_ERR_NOMEM, "device allocation failed");
  }
  int rc = IPMZ_OK;
  if (hipMemcpyAsync(dA, A, (size_t)N * N * 8, hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
    rc = fail(IPMZ_ERR_HIP, "copy-in failed");
  if (!rc) rc = ipmz_bk_factor(ctx, N, dA, N, dp, 0);
  if (rc >= 0 && (hipMemcpy(F, dA, (size_t)N * N * 8, hipMemcpyDeviceToHost) != hipSuccess ||
                  hipMemcpy(ipiv, dp, (size_t)N * 4, hipMemcpyDeviceToHost) != hipSuccess))
    rc = fail(IPMZ_ERR_HIP, "copy-out failed");
  hipFree(dA);
  hipFree(dp);
  return rc < 0 ? rc : IPMZ_OK;  // the reference reports no info
}

int ipmz_overwriting_solve_bunch_kaufman(ipmz_ctx* ctx, int N, const double* F, const int* ipiv, double* b) {
  if (!ctx || N < 0) return fail(IPMZ_ERR_INVALID, "ipmz_overwriting_solve_bunch_kaufman: bad arguments");
  if (N == 0) return IPMZ_OK;
  if (!F || !ipiv || !b) return fail(IPMZ_ERR_INVALID, "null pointer");
  HIP_OK(hipSetDevice(ctx->device));
  double *dF = nullptr, *db = nullptr;
  int* dp = nullptr;
  bool ok = hipMalloc(&dF, (size_t)N * N * 8) == hipSuccess && hipMalloc(&db, (size_t)N * 8) == hipSuccess &&
            hipMalloc(&dp, (size_t)N * 4) == hipSuccess;
  int rc = ok ? IPMZ_OK : fail(IPMZ_ERR_NOMEM, "device allocation failed");
  if (!rc && (hipMemcpyAsync(dF, F, (size_t)N * N * 8, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
              hipMemcpyAsync(db, b, (size_t)N * 8, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
              hipMemcpyAsync(dp, ipiv, (size_t)N * 4, hipMemcpyHostToDevice, ctx->stream) != hipSuccess))
    rc = fail(IPMZ_ERR_HIP, "copy-in failed");
  if (!rc) rc = ipmz_bk_solve(ctx, N, dF, N, dp, db);
  if (!rc && (hipMemcpyAsync(b, db, (size_t)N * 8, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
              hipStreamSynchronize(ctx->stream) != hipSuccess))
    rc = fail(IPMZ_ERR_HIP, "copy-out failed");
  hipFree(dF);
  hipFree(db);
  hipFree(dp);
  return rc;
}

// Host adapters with the reference's signatures ------------------------------
int ipmz_ldlt_decomposition(ipmz_ctx* ctx, int N, const double* A, double* L, double* D) {
  if (!ctx || N < 0 || (N > 0 && (!A || !L || !D))) return fail(IPMZ_ERR_INVALID, "ipmz_ldlt_decomposition: bad arguments");
  if (N == 0) return IPMZ_OK;
  HIP_OK(hipSetDevice(ctx->device));
  const int64_t ld = round_up(N, 64);
  const int64_t wsb = ws_layout(N, nbo_for(ctx, N), ctx->nbi).total;
  double *dK = nullptr, *dD = nullptr;
  char* ws = nullptr;
  HIP_OK(hipMalloc(&dK, (size_t)(ld * N * 8)));
  if (hipMalloc(&dD, (size_t)N * 8) != hipSuccess || hipMalloc(&ws, (size_t)wsb) != hipSuccess) {
    hipFree(dK);
    hipFree(dD);
    return fail(IPMZ_ERR_NOMEM, "device allocation failed");
  }
  int rc = IPMZ_OK;
  if (hipMemcpy2DAsync(dK, ld * 8, A, (size_t)N * 8, (size_t)N * 8, N, hipMemcpyHostToDevice, ctx->stream) !=
      hipSuccess)
    rc = fail(IPMZ_ERR_HIP, "copy-in failed");
  if (!rc) rc = factor_impl(ctx, N, dK, ld, dD, ws, nullptr);
  int info = 0;
  if (!rc) {
    info = read_info(ctx, ws, N);
    if (info < 0) rc = info;
  }
  if (!rc) {
    if (hipMemcpy2D(L, (size_t)N * 8, dK, ld * 8, (size_t)N * 8, N, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(D, dD, (size_t)N * 8, hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail(IPMZ_ERR_HIP, "copy-out failed");
  }
  hipFree(dK);
  hipFree(dD);
  hipFree(ws);
  if (rc) return rc;
  // the reference returns a full L: zeros above, ones on the diagonal (LinearSolvers.cpp:18, :38)
  for (int i = 0; i < N; ++i) {
    L[(int64_t)i * N + i] = 1.0;
    for (int j = i + 1; j < N; ++j) L[(int64_t)i * N + j] = 0.0;
  }
  return info;
}

int ipmz_overwriting_solve_ldlt(ipmz_ctx* ctx, int N, const double* L, const double* D, double* b) {
  if (!ctx || N < 0) return fail(IPMZ_ERR_INVALID, "ipmz_overwriting_solve_ldlt: bad arguments");
  if (N == 0) return IPMZ_OK;  // LinearSolvers.cpp:46-48
  if (!L || !D || !b) return fail(IPMZ_ERR_INVALID, "null pointer");
  HIP_OK(hipSetDevice(ctx->device));
  const int64_t ld = round_up(N, 64);
  const int64_t wsb = ws_layout(N, nbo_for(ctx, N), ctx->nbi).total;
  double *dL = nullptr, *dD = nullptr, *db = nullptr;
  char* ws = nullptr;
  bool ok = hipMalloc(&dL, (size_t)(ld * N * 8)) == hipSuccess && hipMalloc(&dD, (size_t)N * 8) == hipSuccess &&
            hipMalloc(&db, (size_t)N * 8) == hipSuccess && hipMalloc(&ws, (size_t)wsb) == hipSuccess;
  int rc = ok ? IPMZ_OK : fail(IPMZ_ERR_NOMEM, "device allocation failed");
  if (!rc && (hipMemcpy2DAsync(dL, ld * 8, L, (size_t)N * 8, (size_t)N * 8, N, hipMemcpyHostToDevice, ctx->stream) !=
                  hipSuccess ||
              hipMemcpyAsync(dD, D, (size_t)N * 8, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
              hipMemcpyAsync(db, b, (size_t)N * 8, hipMemcpyHostToDevice, ctx->stream) != hipSuccess))
    rc = fail(IPMZ_ERR_HIP, "copy-in failed");
  if (!rc) rc = ipmz_ldlt_prepare_solve(ctx, N, dL, ld, ws, wsb);
  if (!rc) rc = ipmz_ldlt_solve(ctx, N, dL, ld, dD, ws, db);
  // ws is freed below: check the solve's error words now, not at a later sync
  ctx->check_pe = ctx->check_se = nullptr;
  if (!rc) rc = ws_status(ctx->stream, ws, N, nbo_for(ctx, N), ctx->nbi, "ipmz_overwriting_solve_ldlt");
  if (!rc && (hipMemcpyAsync(b, db, (size_t)N * 8, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
              hipStreamSynchronize(ctx->stream) != hipSuccess))
    rc = fail(IPMZ_ERR_HIP, "copy-out failed");
  hipFree(dL);
  hipFree(dD);
  hipFree(db);
  hipFree(ws);
  return rc;
}

}  // extern "C"

// ===========================================================================
// Newton-step solver: B QPs with identical dimensions (B = 1 for ipmz_qp_*).
// Every per-QP array lives in one allocation with a per-QP stride; the
// kernels take a device array of QPDev descriptors and index it with
// blockIdx.y, so one launch serves the whole batch.
struct ipmz_qp {
  ipmz_ctx* ctx = nullptr;
  int n = 0, m = 0, p = 0, N = 0, B = 1;
  int64_t ldn = 0, ldk = 0, state_len = 0;
  double delta = 1e-4;
  std::vector<void*> allocs;
  std::vector<QPDev> hq;   // host copies of the descriptors
  QPDev* dq = nullptr;     // device array of B descriptors
  QPBatch qb{};
  // factor storage
  double *K = nullptr, *D = nullptr;
  int64_t sK = 0, sD = 0, sb = 0;
  // batches of small systems (fused phases, LDL^T): the assembled KKT kept
  // across steps (off-diagonal part written once per data load, the diagonal
  // every step); the small factor reads it and writes L to K (strides sK)
  double* K0 = nullptr;
  char* ws = nullptr;      // B == 1: ws_layout(N) ; B > 1: see batch_ws
  int64_t ws_bytes = 0;
  double *bLinv = nullptr, *bW = nullptr;  // batched factor workspace (B > 1)
  int* binfo = nullptr;
  int64_t sL = 0, sW = 0;
  bool loaded = false;
  // mixed precision (C5): fp32 factor of S K S + fp64 refinement
  bool mixed = false;
  double ir_tol = 1e-12;
  int ir_max = 10;
  MixedWs mw;
  char* mws = nullptr;
  // normal-equations reduction (C2)
  bool normal = false;
  // EqualityHandling::None: Bunch-Kaufman factor (pivots per QP)
  bool eqnone = false;
  char* bkws = nullptr;  // the whole-device Bunch-Kaufman factor's workspace (B == 1, N >= IPMZ_BK_GRID_MIN)
  double* bklt = nullptr;  // its factor transposed (N x N): the interchange folding's input, the fallback's factor
  char* bkfws = nullptr;   // the device-wide solve's workspace (bk_ws), L' in K
  unsigned* pflags = nullptr;  // B > 1: the two-workgroup small factor's flags + sticky error word
  int small_kernel = IPMZ_BATCH_FACTOR_AUTO;  // ipmz_batch_set_factor_kernel
  bool eqpen = false;  // EqualityHandling::PenaltyFunction (LDL^T)
  // InequalityHandling / Bounds (which Newton slots exist)
  bool slacks = false, naive = false;
  // EqualityHandling::SlackedSlacks: m, p below are the step's (m + p equality
  // rows run as l = u = d inequalities, p = 0); m_usr, p_usr the data's
  bool eqss = false;
  int m_usr = 0, p_usr = 0;
  bool vlo = true, vup = true, alo = true, aup = true;
  int* ipiv = nullptr;
  int64_t sP = 0;
  char* nws = nullptr;
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec = nullptr;
  int graph_flags = -1;
  // timing
  bool timing = false;
  std::vector<hipEvent_t> ev;  // phase boundary events
  hipEvent_t (*tr_pairs)[2] = nullptr;
  // completion of the last multi-stream (eager) step: the next one is not
  // enqueued before it (queue depth 1, see step_impl)
  hipEvent_t step_done = nullptr;
  hipEvent_t step_in = nullptr;  // the caller's stream reached the step (the fork onto ctx->own)
  bool step_pending = false;
  int last_step_graph = 0;  // the last ipmz_qp_step replayed a captured hipGraph
  int tr_cap = 0;
  double ph_ms[IPMZ_PH_COUNT] = {0};
  double tr_flops = 0.0;
  int64_t tr_launches = 0;
};

namespace {
// Newton variables present per formulation (SymbolicOptimization.cpp
// get_variables_: absent blocks are dropped from the Newton order)
int64_t slot_len(const ipmz_qp* s, int slot) {
  switch (slot) {
    case X: return s->n;
    case LY: return s->vlo ? s->n : 0;
    case LZ: return s->vup ? s->n : 0;
    case Y: return (s->vlo && !s->slacks) ? s->n : 0;
    case Z: return (s->vup && !s->slacks) ? s->n : 0;
    case LA: case S: return s->naive ? 0 : s->m;
    case LG: return s->alo ? s->m : 0;
    case LH: return s->aup ? s->m : 0;
    case G: return (s->alo && !s->slacks) ? s->m : 0;
    case H: return (s->aup && !s->slacks) ? s->m : 0;
    case P: return (s->eqnone || s->eqpen) ? 0 : s->p;
    default: return s->p;
  }
}

// one allocation of B x stride doubles (stride = per-QP count rounded to 64 B)
double* dev_array(ipmz_qp* s, int64_t count, int64_t* stride_out = nullptr) {
  const int64_t stride = round_up(count < 1 ? 1 : count, 8);
  void* ptr = nullptr;
  if (hipMalloc(&ptr, (size_t)(stride * s->B) * sizeof(double)) != hipSuccess) return nullptr;
  s->allocs.push_back(ptr);
  if (stride_out) *stride_out = stride;
  return static_cast<double*>(ptr);
}

// slot pointers into one contiguous Newton-order vector (the reference's
// order; NaiveSlacks puts its duals lambda_g, lambda_h ahead of lambda_C,
// formulations.txt)
void carve(const ipmz_qp* s, double* base, double** slots) {
  static const int naive_order[NSLOT] = {X, LG, LH, LC, P, LY, LZ, G, H, Y, Z, LA, S};
  int64_t off = 0;
  for (int k = 0; k < NSLOT; ++k) {
    const int slot = s->naive ? naive_order[k] : k;
    slots[slot] = base + off;
    off += slot_len(s, slot);
  }
}

QPDev& q0(ipmz_qp* s) { return s->hq[0]; }

int solve_batch(ipmz_qp* s, hipStream_t st, int which) {
  if (s->eqnone && s->bkfws) {  // overwriting_solve_bunch_kaufman, device-wide (L' in K)
    HIP_OK(bk_run(s->K, s->ldk, s->N, s->bklt, s->ipiv, bk_ws(s->bkfws, s->N), q0(s).b, st));
  } else if (s->eqnone && s->bklt) {  // overwriting_solve_bunch_kaufman on the transposed factor
    HIP_OK(bk_solve_lt(s->bklt, s->N, s->ipiv, q0(s).b, st));
  } else if (s->eqnone) {  // overwriting_solve_bunch_kaufman
    HIP_OK(bk_solve(s->K, s->ldk, s->N, s->ipiv, q0(s).b, s->B, s->sK, s->sP, s->sb, st));
  } else if (s->normal) {
    return normal_solve_impl(s->ctx, s->n, s->m + s->p, s->K, s->ldk, s->D,
                             normal_ws(s->nws, s->n, s->m + s->p, s->ctx), q0(s).b);
  } else if (s->mixed) {
    HIP_OK(mixed_solve(s->K, s->ldk, s->mw, q0(s).b, s->ir_tol, s->ir_max, st));
    HIP_OK(hipMemcpyAsync(q0(s).scal + IPMZ_SC_IR_RATIO_AFF + 2 * which, s->mw.stat, 2 * sizeof(double),
                          hipMemcpyDeviceToDevice, st));
  } else if (s->B == 1) {
    HIP_OK(solve_ws(s->K, s->ldk, s->N, s->D, s->ws, nbo_for(s->ctx, s->N), s->ctx->nbi, q0(s).b, st));
  } else {
    HIP_OK(ldlt_solve_batched(s->K, s->ldk, s->N, s->D, s->bLinv, s->ctx->nbi, q0(s).b, s->B, s->sK, s->sD, s->sL,
                              s->sb, st));
  }
  return IPMZ_OK;
}

// info_reset: the caller already reset the batched factor's info word
bool uses_k0(const ipmz_qp* s);
int factor_batch(ipmz_qp* s, TrailTimer* tt, bool info_reset) {
  if (s->eqnone) {  // zero diagonal block: symmetric_indefinite_factorization (reference kp behaviour)
    if (s->bkws) {
      HIP_OK(bk_factor_grid(s->K, s->ldk, s->N, s->ipiv, s->binfo, 0, s->bkws, s->ctx->stream));
      HIP_OK(bk_transpose(s->K, s->ldk, s->N, s->bklt, s->ctx->stream));
      if (s->bkfws)  // L' into K (the factor is not read again this step)
        HIP_OK(bk_setup(s->K, s->ldk, s->N, s->ipiv, s->binfo, s->bklt, s->K, s->ldk, bk_ws(s->bkfws, s->N),
                        s->ctx->stream));
      return IPMZ_OK;
    }
    HIP_OK(bk_factor(s->K, s->ldk, s->N, s->ipiv, s->binfo, 0, s->B, s->sK, s->sP, s->ctx->stream));
    return IPMZ_OK;
  }
  if (s->mixed) return mixed_factor_impl(s->ctx, s->K, s->ldk, s->mw, tt);
  if (s->normal)
    return normal_factor_impl(s->ctx, s->n, s->m + s->p, s->K, s->ldk, s->D,
                              normal_ws(s->nws, s->n, s->m + s->p, s->ctx), tt);
  if (s->B == 1) return factor_impl(s->ctx, s->N, s->K, s->ldk, s->D, s->ws, tt);
  BatchStrides bs;
  bs.B = s->B;
  bs.sK = s->sK;
  bs.sD = s->sD;
  bs.sL = s->sL;
  bs.sW = s->sW;
  bs.pflags = s->pflags;
  bs.small_kernel = s->small_kernel;
  bs.K0 = info_reset && uses_k0(s) ? s->K0 : nullptr;  // (info_reset: the fused step, whose pre phase assembled into K0)
  if (!info_reset) HIP_OK(hipMemsetAsync(s->binfo, 0x7f, sizeof(int), s->ctx->stream));
  HIP_OK(ldlt_factor_batched(s->K, s->ldk, s->N, s->D, s->bLinv, s->bW, nbo_for(s->ctx, s->N), s->ctx->nbi, s->binfo,
                             s->ctx->stream, bs));
  return IPMZ_OK;
}

// batches of small systems: the O(N) / O(n^2) phases as three per-QP
// workgroup kernels (newton.hip k_fused_*)
bool fused_phases(const ipmz_qp* s) { return s->B > 1 && s->N <= IPMZ_FUSED_NMAX; }
// ... whose solves are the small batched solve (solve_batch's last branch,
// nbi 64): then both solves and the phases between them run as one launch
bool fused_solves(const ipmz_qp* s) {
  return fused_phases(s) && !s->eqnone && !s->normal && !s->mixed && s->ctx->nbi == 64 && fused_solves_ok(s->N, s->ldk) &&
         !(debug_inject_mask() & IPMZ_DEBUG_NO_FUSED_SOLVES);
}
// the fused step keeps the assembled matrix in K0 when the small batched
// factor (nbi 64) consumes it; otherwise the whole matrix is assembled into K
bool uses_k0(const ipmz_qp* s) {
  return s->K0 && s->ctx->nbi == 64 && s->N <= IPMZ_SMALL_NMAX && !(debug_inject_mask() & IPMZ_DEBUG_NO_K0);
}

int run_step(ipmz_qp* s, int flags) {
  hipStream_t st = s->ctx->stream;
  const QPBatch& qb = s->qb;
  const bool t = s->timing;
  auto mark = [&](int i) {
    IPMZ_TRACE("step: phase mark %d", i);
    if (t) hipEventRecord(s->ev[i], st);
  };
  const bool restart = flags & IPMZ_STEP_RESTART_IF_CONVERGED;
  const int freeze = restart ? 0 : 1;
  const bool fused = fused_phases(s);
  TrailTimer tt;
  tt.pairs = s->tr_pairs;
  tt.cap = t ? s->tr_cap : 0;
  int rc;
  if (fused) {
    // phases: assemble = pre (restart, assembly, affine rhs); factor;
    // solve = the two solves; eval = mid + post
    mark(0);
    HIP_OK(qp_fused_pre(qb, restart ? 1 : 0, s->eqnone ? nullptr : s->binfo, st, uses_k0(s) ? KMODE_K0_DIAG : KMODE_K));
    mark(1);
    if ((rc = factor_batch(s, nullptr, true))) return rc;
    mark(2);
    if (fused_solves(s)) {
      // both solves and the phases between them in one launch (the solve
      // phase then holds mid and post too; eval = the evaluation alone)
      HIP_OK(qp_fused_solves(qb, s->K, s->ldk, s->N, s->D, s->bLinv, q0(s).b, s->sK, s->sD, s->sL, s->sb, freeze, st));
      mark(3);
      mark(4);
      mark(5);
      HIP_OK(qp_fused_eval(qb, st));
    } else {
      if ((rc = solve_batch(s, st, 0))) return rc;
      mark(3);
      HIP_OK(qp_fused_mid(qb, st));
      mark(4);
      if ((rc = solve_batch(s, st, 1))) return rc;
      mark(5);
      HIP_OK(qp_fused_post(qb, freeze, st));
    }
    mark(6);
    mark(7);
  } else {
    if (restart) HIP_OK(qp_restart_if_converged(qb, st));
    mark(0);
    HIP_OK(qp_assemble(qb, st));
    mark(1);
    if ((rc = factor_batch(s, t ? &tt : nullptr, false))) return rc;
    mark(2);
    // predictor (affine scaling) direction
    HIP_OK(qp_rhs(qb, st));
    if ((rc = solve_batch(s, st, 0))) return rc;
    mark(3);
    HIP_OK(qp_backsub(qb, 0, st));
    HIP_OK(qp_ratio(qb, 0, SC_ALPHA_AFF, st));
    HIP_OK(qp_mu_aff(qb, st));
    // centering-corrector direction
    HIP_OK(qp_corrector_residuals(qb, st));
    HIP_OK(qp_rhs(qb, st));
    mark(4);
    if ((rc = solve_batch(s, st, 1))) return rc;
    mark(5);
    HIP_OK(qp_backsub(qb, 1, st));
    HIP_OK(qp_ratio(qb, 1, SC_ALPHA, st));
    HIP_OK(qp_update(qb, freeze, st));
    mark(6);
    HIP_OK(qp_evaluate(qb, st));
    mark(7);
  }
  if (t) {
    HIP_OK(hipStreamSynchronize(st));
    float ms = 0.f;
    auto el = [&](int a, int b) {
      hipEventElapsedTime(&ms, s->ev[a], s->ev[b]);
      return (double)ms;
    };
    s->ph_ms[IPMZ_PH_STEP] += el(0, 7);
    s->ph_ms[IPMZ_PH_ASSEMBLE] += el(0, 1);
    s->ph_ms[IPMZ_PH_FACTOR] += el(1, 2);
    s->ph_ms[IPMZ_PH_SOLVE] += el(2, 3) + el(4, 5);
    s->ph_ms[IPMZ_PH_EVAL] += fused ? el(3, 4) + el(5, 6) : el(6, 7);
    for (int i = 0; i < tt.used; ++i) {
      hipEventElapsedTime(&ms, s->tr_pairs[i][0], s->tr_pairs[i][1]);
      s->ph_ms[IPMZ_PH_TRAILING] += ms;
    }
    s->tr_launches += tt.used;
    s->tr_flops += tt.flops * s->B;
  }
  return IPMZ_OK;
}

int evaluate_and_save(ipmz_qp* s) {
  hipStream_t st = s->ctx->stream;
  if (s->K0) HIP_OK(qp_fused_pre(s->qb, 0, nullptr, st, KMODE_K0_OFFDIAG));  // the data just changed
  HIP_OK(qp_evaluate(s->qb, st));
  HIP_OK(qp_save_initial(s->qb, st));
  s->loaded = true;
  return IPMZ_OK;
}

int create_solver(ipmz_ctx* ctx, const ipmz_qp_config* cfg, int B, ipmz_qp** out) {
  if (!ctx || !cfg || !out) return fail(IPMZ_ERR_INVALID, "null argument");
  *out = nullptr;
  if (cfg->n <= 0 || cfg->m < 0 || cfg->p < 0 || B <= 0)
    return fail(IPMZ_ERR_INVALID, "dimensions: n > 0, m >= 0, p >= 0, batch > 0");
  if (cfg->equality_handling != IPMZ_EQ_REGULARIZATION && cfg->equality_handling != IPMZ_EQ_NONE &&
      cfg->equality_handling != IPMZ_EQ_PENALTY && cfg->equality_handling != IPMZ_EQ_PENALTY_EXTRA_DUAL &&
      cfg->equality_handling != IPMZ_EQ_SLACKED_SLACKS && cfg->equality_handling != IPMZ_EQ_NAIVE_SLACKS)
    return fail(IPMZ_ERR_INVALID, "unknown equality handling");
  const int mk = cfg->inequality_handling == IPMZ_INEQ_NAIVE_SLACKS ? 2 * cfg->m : cfg->m;
  if (cfg->equality_handling == IPMZ_EQ_NONE && B > 1 && cfg->n + mk + cfg->p > IPMZ_BK_NMAX)
    return fail(IPMZ_ERR_INVALID, "EqualityHandling::None in batches factors with Bunch-Kaufman one workgroup per "
                                  "system: N <= " + std::to_string(IPMZ_BK_NMAX));
  const int ih = cfg->inequality_handling, ib = cfg->inequality_bounds, vb = cfg->variable_bounds;
  if (ih != IPMZ_INEQ_SLACKED_SLACKS && ih != IPMZ_INEQ_SLACKS && ih != IPMZ_INEQ_NAIVE_SLACKS)
    return fail(IPMZ_ERR_INVALID, "unknown inequality handling");
  if (ih == IPMZ_INEQ_NAIVE_SLACKS && cfg->m > 0 && ib != IPMZ_BOUNDS_BOTH)
    return fail(IPMZ_ERR_INVALID, "InequalityHandling::NaiveSlacks: both inequality bounds");
  if (cfg->equality_handling == IPMZ_EQ_NAIVE_SLACKS && (ih != IPMZ_INEQ_NAIVE_SLACKS || ib != IPMZ_BOUNDS_BOTH))
    return fail(IPMZ_ERR_INVALID, "EqualityHandling::NaiveSlacks: with InequalityHandling::NaiveSlacks and both "
                                  "inequality bounds");
  if (cfg->equality_handling == IPMZ_EQ_SLACKED_SLACKS && (ih != IPMZ_INEQ_SLACKED_SLACKS || ib != IPMZ_BOUNDS_BOTH))
    return fail(IPMZ_ERR_INVALID, "EqualityHandling::SlackedSlacks: with InequalityHandling::SlackedSlacks and both "
                                  "inequality bounds");
  if (ib < IPMZ_BOUNDS_BOTH || ib > IPMZ_BOUNDS_NONE || vb < IPMZ_BOUNDS_BOTH || vb > IPMZ_BOUNDS_NONE)
    return fail(IPMZ_ERR_INVALID, "unknown bounds setting");
  if (cfg->m > 0 && ib == IPMZ_BOUNDS_NONE)
    return fail(IPMZ_ERR_INVALID, "inequality rows need a lower or an upper bound (inequality_bounds != NONE)");
  if (ih == IPMZ_INEQ_SLACKS && ((cfg->m > 0 && ib != IPMZ_BOUNDS_BOTH) || vb != IPMZ_BOUNDS_BOTH))
    return fail(IPMZ_ERR_INVALID, "InequalityHandling::Slacks is built on both bounds (the reference's Slacks "
                                  "formulation drops one-sided bounds inconsistently)");
  HIP_OK(hipSetDevice(ctx->device));
  auto* s = new ipmz_qp();
  s->ctx = ctx;
  {
    std::lock_guard<std::mutex> lk(g_ctx_mutex);
    if (ctx->closed) {
      delete s;
      return fail(IPMZ_ERR_STATE, "context already destroyed");
    }
    ++ctx->users;
  }
  s->B = B;
  s->n = cfg->n;
  s->m_usr = cfg->m;
  s->p_usr = cfg->p;
  // equality SlackedSlacks / NaiveSlacks: the p rows appended to the
  // inequality block of the same handling with l = u = d
  s->eqss = cfg->equality_handling == IPMZ_EQ_SLACKED_SLACKS || cfg->equality_handling == IPMZ_EQ_NAIVE_SLACKS;
  s->m = s->eqss ? cfg->m + cfg->p : cfg->m;
  s->p = s->eqss ? 0 : cfg->p;
  s->N = cfg->equality_handling == IPMZ_EQ_NAIVE_SLACKS ? cfg->n + 2 * (cfg->m + cfg->p) : cfg->n + mk + cfg->p;
  s->delta = cfg->delta > 0 ? cfg->delta : 1e-4;
  s->eqnone = cfg->equality_handling == IPMZ_EQ_NONE;
  s->eqpen = cfg->equality_handling == IPMZ_EQ_PENALTY || cfg->equality_handling == IPMZ_EQ_PENALTY_EXTRA_DUAL;
  s->slacks = ih == IPMZ_INEQ_SLACKS;
  s->naive = ih == IPMZ_INEQ_NAIVE_SLACKS;
  s->vlo = vb == IPMZ_BOUNDS_BOTH || vb == IPMZ_BOUNDS_LOWER;
  s->vup = vb == IPMZ_BOUNDS_BOTH || vb == IPMZ_BOUNDS_UPPER;
  s->alo = ib == IPMZ_BOUNDS_BOTH || ib == IPMZ_BOUNDS_LOWER;
  s->aup = ib == IPMZ_BOUNDS_BOTH || ib == IPMZ_BOUNDS_UPPER;
  s->ldn = round_up(s->n, 8);
  s->ldk = round_up(s->N, 64);
  s->state_len = 0;
  for (int k = 0; k < NSLOT; ++k) s->state_len += slot_len(s, k);
  const int n = s->n, m = s->m, p = s->p, N = s->N;
  int64_t sQ, sA, sC, sn, sm, sp, sS, sNb, sScal, sPart, sT;
  double* Q = dev_array(s, (int64_t)n * s->ldn, &sQ);
  double* A = dev_array(s, (int64_t)m * s->ldn, &sA);
  double* C = dev_array(s, (int64_t)p * s->ldn, &sC);  // (eqss: C is rows m_usr.. of A)
  double* c = dev_array(s, n, &sn);
  double* lx = dev_array(s, n);
  double* ux = dev_array(s, n);
  double* Qx = dev_array(s, n);
  double* ATl = dev_array(s, n);
  double* CTl = dev_array(s, n);
  double* lA = dev_array(s, m, &sm);
  double* uA = dev_array(s, m);
  double* Ax = dev_array(s, m);
  double* d = dev_array(s, s->p_usr, &sp);
  double* Cx = dev_array(s, p);
  double* v = dev_array(s, s->state_len, &sS);
  double* r = dev_array(s, s->state_len);
  double* da = dev_array(s, s->state_len);
  double* di = dev_array(s, s->state_len);
  double* v0 = dev_array(s, s->state_len);
  double* r0 = dev_array(s, s->state_len);
  double* bvec = dev_array(s, N, &sNb);
  double* scal = dev_array(s, SC_COUNT, &sScal);
  double* scal0 = dev_array(s, SC_COUNT);
  double* part = dev_array(s, 4 * 1024, &sPart);
  double* tpart = dev_array(s, (int64_t)((m > p ? m : p) + IPMZ_TCHUNK - 1) / IPMZ_TCHUNK * n + 8, &sT);
  int64_t sDone;
  double* done = dev_array(s, 1, &sDone);
  s->K = dev_array(s, (int64_t)N * s->ldk, &s->sK);
  if (B > 1 && N <= IPMZ_FUSED_NMAX && !s->eqnone) {
    int64_t sK0 = 0;
    s->K0 = dev_array(s, (int64_t)N * s->ldk, &sK0);
  }
  s->D = dev_array(s, N, &s->sD);
  s->sb = sNb;
  bool ok = Q && A && C && c && lx && ux && Qx && ATl && CTl && lA && uA && Ax && d && Cx && v && r && da && di &&
            v0 && r0 && bvec && scal && scal0 && part && tpart && done && s->K && s->D &&
            hipMemset(done, 0, (size_t)(sDone * B) * sizeof(double)) == hipSuccess;
  if (ok && B == 1) {
    s->ws_bytes = ws_layout(N, nbo_for(ctx, N), ctx->nbi).total;
    void* w = nullptr;
    ok = hipMalloc(&w, (size_t)s->ws_bytes) == hipSuccess && hipMemset(w, 0, (size_t)s->ws_bytes) == hipSuccess;
    if (ok) s->allocs.push_back(w);
    s->ws = static_cast<char*>(w);
  } else if (ok) {
    const int64_t nblk = (N + ctx->nbi - 1) / ctx->nbi;
    s->bLinv = dev_array(s, nblk * ctx->nbi * ctx->nbi, &s->sL);
    s->bW = dev_array(s, (int64_t)N * nbo_for(ctx, N), &s->sW);
    void* w = nullptr;
    ok = s->bLinv && s->bW && hipMalloc(&w, (size_t)(B * 4 > 256 ? B * 4 : 256)) == hipSuccess;  // one info per QP
    if (ok) s->allocs.push_back(w);
    s->binfo = static_cast<int*>(w);
    if (ok) {  // flags of the two-workgroup small factor (B <= #CU)
      ok = hipMalloc(&w, ((size_t)B * IPMZ_PAIR_FLAGS + 1) * sizeof(unsigned)) == hipSuccess &&
           hipMemset(w, 0, ((size_t)B * IPMZ_PAIR_FLAGS + 1) * sizeof(unsigned)) == hipSuccess;
      if (ok) s->allocs.push_back(w);
      s->pflags = static_cast<unsigned*>(w);
    }
  }
  if (ok && s->eqnone) {
    s->sP = round_up(N, 16);
    void* w = nullptr;
    ok = hipMalloc(&w, (size_t)(s->sP * B) * sizeof(int)) == hipSuccess;
    if (ok) s->allocs.push_back(w);
    s->ipiv = static_cast<int*>(w);
    if (ok && !s->binfo) {
      ok = hipMalloc(&w, 256) == hipSuccess;
      if (ok) s->allocs.push_back(w);
      s->binfo = static_cast<int*>(w);
    }
    if (ok && B == 1 && N >= IPMZ_BK_GRID_MIN) {
      ok = hipMalloc(&w, bk_grid_ws_bytes(N)) == hipSuccess;
      if (ok) s->allocs.push_back(w);
      s->bkws = static_cast<char*>(w);
      if (ok) ok = hipMalloc(&w, (size_t)N * N * sizeof(double)) == hipSuccess;
      if (ok) s->allocs.push_back(w);
      s->bklt = static_cast<double*>(w);
      const int64_t bkb = bk_ws(nullptr, N).total;
      if (ok) ok = hipMalloc(&w, (size_t)bkb) == hipSuccess && hipMemset(w, 0, (size_t)bkb) == hipSuccess;
      if (ok) s->allocs.push_back(w);
      s->bkfws = static_cast<char*>(w);
    }
  }
  if (!ok) {
    ipmz_qp_destroy(s);
    return fail(IPMZ_ERR_NOMEM, "device allocation failed");
  }
  s->hq.resize(B);
  for (int i = 0; i < B; ++i) {
    QPDev& q = s->hq[i];
    q = QPDev{};
    q.n = n;
    q.m = m;
    q.p = p;
    q.N = N;
    q.ldn = s->ldn;
    q.ldk = s->ldk;
    q.state_len = s->state_len;
    q.delta = s->delta;
    q.eqnone = s->eqnone ? 1 : 0;
    q.eqpen = s->eqpen ? 1 : 0;
    q.slacks = s->slacks ? 1 : 0;
    q.naive = s->naive ? 1 : 0;
    q.eqss = s->eqss ? 1 : 0;
    q.m_usr = s->m_usr;
    q.p_usr = s->p_usr;
    q.mk = s->naive ? 2 * m : m;
    q.vlo = s->vlo ? 1 : 0;
    q.vup = s->vup ? 1 : 0;
    q.alo = s->alo ? 1 : 0;
    q.aup = s->aup ? 1 : 0;
    q.Q = Q + i * sQ;
    q.A = A + i * sA;
    q.C = s->eqss ? q.A + (int64_t)s->m_usr * s->ldn : C + i * sC;
    q.c = c + i * sn;
    q.lx = lx + i * sn;
    q.ux = ux + i * sn;
    q.Qx = Qx + i * sn;
    q.ATl = ATl + i * sn;
    q.CTl = CTl + i * sn;
    q.lA = lA + i * sm;
    q.uA = uA + i * sm;
    q.Ax = Ax + i * sm;
    q.d = d + i * sp;
    q.Cx = Cx + i * sp;
    carve(s, v + i * sS, q.v);
    carve(s, r + i * sS, q.r);
    carve(s, da + i * sS, q.daff);
    carve(s, di + i * sS, q.dir);
    q.v0 = v0 + i * sS;
    q.r0 = r0 + i * sS;
    q.b = bvec + i * sNb;
    q.scal = scal + i * sScal;
    q.scal0 = scal0 + i * sScal;
    q.part = part + i * sPart;
    q.tpart = tpart + i * sT;
    q.K = s->K + i * s->sK;
    q.K0 = s->K0 ? s->K0 + i * s->sK : nullptr;
    q.done = reinterpret_cast<unsigned*>(done + i * sDone);
  }
  void* dqp = nullptr;
  if (hipMalloc(&dqp, sizeof(QPDev) * B) != hipSuccess) {
    ipmz_qp_destroy(s);
    return fail(IPMZ_ERR_NOMEM, "device allocation failed");
  }
  s->allocs.push_back(dqp);
  s->dq = static_cast<QPDev*>(dqp);
  HIP_OK(hipMemcpy(s->dq, s->hq.data(), sizeof(QPDev) * B, hipMemcpyHostToDevice));
  s->qb = QPBatch{s->dq, s->hq[0], B};
  HIP_OK(hipMemsetAsync(scal, 0, (size_t)sScal * B * 8, ctx->stream));
  HIP_OK(hipMemsetAsync(s->K, 0, (size_t)s->sK * B * 8, ctx->stream));
  HIP_OK(hipStreamSynchronize(ctx->stream));
  *out = s;
  return IPMZ_OK;
}

int check_index(ipmz_qp* s, int i) {
  if (!s || i < 0 || i >= s->B) return fail(IPMZ_ERR_INVALID, "QP index out of range");
  return IPMZ_OK;
}

int load_one(ipmz_qp* s, int i, const double* Q, const double* c, const double* A, const double* lA, const double* uA,
             const double* C, const double* d, const double* lx, const double* ux) {
  if (!Q || !c || !lx || !ux || (s->m_usr && (!A || !lA || !uA)) || (s->p_usr && (!C || !d)))
    return fail(IPMZ_ERR_INVALID, "load: missing data block");
  // EnvironmentBuilder.cpp:12-17 (the reference ASSERTs; here an error code)
  for (int k = 0; k < s->n; ++k)
    if (!(lx[k] < ux[k])) return fail(IPMZ_ERR_INVALID, "l_x < u_x violated at " + std::to_string(k));
  for (int k = 0; k < s->m_usr; ++k)
    if (!(lA[k] <= uA[k])) return fail(IPMZ_ERR_INVALID, "l_A <= u_A violated at " + std::to_string(k));
  HIP_OK(hipSetDevice(s->ctx->device));
  hipStream_t st = s->ctx->stream;
  const QPDev& q = s->hq[i];
  const size_t rowb = (size_t)s->n * 8, ldb = (size_t)s->ldn * 8;
  HIP_OK(hipMemcpy2DAsync((void*)q.Q, ldb, Q, rowb, rowb, s->n, hipMemcpyHostToDevice, st));
  if (s->m_usr) HIP_OK(hipMemcpy2DAsync((void*)q.A, ldb, A, rowb, rowb, s->m_usr, hipMemcpyHostToDevice, st));
  if (s->p_usr) HIP_OK(hipMemcpy2DAsync((void*)q.C, ldb, C, rowb, rowb, s->p_usr, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync((void*)q.c, c, rowb, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync((void*)q.lx, lx, rowb, hipMemcpyHostToDevice, st));
  HIP_OK(hipMemcpyAsync((void*)q.ux, ux, rowb, hipMemcpyHostToDevice, st));
  if (s->m_usr) {
    HIP_OK(hipMemcpyAsync((void*)q.lA, lA, (size_t)s->m_usr * 8, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync((void*)q.uA, uA, (size_t)s->m_usr * 8, hipMemcpyHostToDevice, st));
  }
  if (s->p_usr) HIP_OK(hipMemcpyAsync((void*)q.d, d, (size_t)s->p_usr * 8, hipMemcpyHostToDevice, st));
  if (s->eqss && s->p_usr) {  // the equality rows as l = u = d
    HIP_OK(hipMemcpyAsync((void*)(q.lA + s->m_usr), d, (size_t)s->p_usr * 8, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync((void*)(q.uA + s->m_usr), d, (size_t)s->p_usr * 8, hipMemcpyHostToDevice, st));
  }
  HIP_OK(hipStreamSynchronize(st));
  return IPMZ_OK;
}

// Does the step's factorization fork onto the look-ahead streams?  Such a
// step is enqueued eagerly even when IPMZ_STEP_GRAPH is asked for: its graph
// replay is slower than the eager launches (tools/graph_ab.py, profiles/r03_s3:
// C2 2.4-3.0 vs 1.75 ms, C3 16.7 vs 14.6, C5 35.3 vs 25.7 ms per step -- the
// replayed look-ahead loses its stream priorities and overlap), and a
// multi-millisecond step hides its launch latency anyway.  The capture itself
// is correct (debug bit IPMZ_INJECT_GRAPH_FORKS; tests/test_gpu_graph.py:
// bitwise the eager step): it once crashed inside hipStreamEndCapture of the
// HIP runtime torch bundles, fixed by ldlt.hip's stream_record / stream_wait.
bool step_forks(const ipmz_qp* s) {
  if (s->eqnone || s->B > 1) return false;
  if (debug_inject_mask() & IPMZ_INJECT_GRAPH_FORKS) return false;
  // the augmented factor and the normal equations' pipelined factor are both
  // one factor_impl of order N (= n + m + p): it forks from 3 outer panels
  return (s->N + nbo_for(s->ctx, s->N) - 1) / nbo_for(s->ctx, s->N) >= 3;
}

int step_impl(ipmz_qp* s, int flags) {
  if (!s || !s->loaded) return fail(IPMZ_ERR_STATE, "load or generate the QP first");
  HIP_OK(hipSetDevice(s->ctx->device));
  s->last_step_graph = 0;
  {
    // The caller's stream is capturing (torch.cuda.graph around step()): the
    // whole step goes into the caller's capture on that stream -- no hop to
    // the own stream, no host wait, no nested capture (the look-ahead
    // streams order through capture dependencies, ldlt.hip stream_wait; the
    // mixed solve enqueues all its passes, mixed.hip)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIP_OK(hipStreamIsCapturing(s->ctx->stream, &cs));
    if (cs != hipStreamCaptureStatusNone) {
      if (s->timing) return fail(IPMZ_ERR_STATE, "phase timing inside a caller's graph capture");
      set_capture_origin(s->ctx->stream);
      const int rc = run_step(s, flags & ~IPMZ_STEP_GRAPH);
      set_capture_origin(nullptr);
      return rc;
    }
  }
  if (step_forks(s) && (!s->timing || s->ctx->stream != s->ctx->own)) {  // timing: phase events on own, below
    // A factorization that forks onto the look-ahead streams is enqueued
    // eagerly (~130-160 launches and event waits over four queues); with
    // the next step's packets already queued behind it the command processor
    // slows the running step down (C2: 3.9 vs 3.1 ms per step back to back;
    // tools/step_sync_ab.py), so at most one such step is in flight: the host
    // waits for the previous one before enqueuing the next.
    if (!s->step_done) HIP_OK(hipEventCreateWithFlags(&s->step_done, hipEventDisableTiming));
    if (s->step_pending) HIP_OK(hipEventSynchronize(s->step_done));
    s->step_pending = false;
    // On a stream the caller made (torch's default or side streams) the step
    // runs on the context's own stream, forked from the caller's, and the host
    // waits for it before the caller's stream is joined to it: a join left
    // pending on the caller's stream while the step runs cost ~1.2 ms per C3
    // step (15.7 vs 14.5 ms; the step on the caller's stream itself the same),
    // profiles/r03_s5/origin_stream_ab.log.  The host would wait for the step
    // before enqueuing the next one anyway (queue depth 1).
    hipStream_t caller = s->ctx->stream, own = s->ctx->own;
    const bool hop = caller != own;
    if (hop) {
      if (!s->step_in) HIP_OK(hipEventCreateWithFlags(&s->step_in, hipEventDisableTiming));
      HIP_OK(hipEventRecord(s->step_in, caller));
      HIP_OK(hipStreamWaitEvent(own, s->step_in, 0));
      s->ctx->stream = own;
    }
    const int rc = run_step(s, flags);
    s->ctx->stream = caller;
    if (rc) return rc;
    HIP_OK(hipEventRecord(s->step_done, own));
    if (hop) {
      HIP_OK(hipEventSynchronize(s->step_done));
      HIP_OK(hipStreamWaitEvent(caller, s->step_done, 0));  // complete: orders nothing pending
      return IPMZ_OK;
    }
    s->step_pending = true;
    return IPMZ_OK;
  }
  if (!(flags & IPMZ_STEP_GRAPH) || s->timing) return run_step(s, flags);
  hipStream_t st = s->ctx->stream;
  if (!s->gexec || s->graph_flags != flags) {
    if (s->gexec) hipGraphExecDestroy(s->gexec);
    if (s->graph) hipGraphDestroy(s->graph);
    s->gexec = nullptr;
    s->graph = nullptr;
    // capture on the context's own stream: the caller's stream may be the
    // legacy default stream (torch's), which cannot be captured; the graph
    // is then launched on the caller's stream
    hipStream_t cap = s->ctx->own;
    IPMZ_TRACE("capture: begin");
    set_capture_origin(cap);  // ldlt.hip stream_wait: the look-ahead streams' ordering inside the capture
    HIP_OK(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
    s->ctx->stream = cap;
    int rc = run_step(s, flags);
    s->ctx->stream = st;
    IPMZ_TRACE("capture: step enqueued rc=%d", rc);
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(cap, &g);
    set_capture_origin(nullptr);
    IPMZ_TRACE("capture: ended %d", (int)e);
    if (rc) {
      if (g) hipGraphDestroy(g);
      return rc;
    }
    if (e != hipSuccess) return fail(IPMZ_ERR_HIP, std::string("graph capture: ") + hipGetErrorString(e));
    s->graph = g;
    HIP_OK(hipGraphInstantiate(&s->gexec, g, nullptr, nullptr, 0));
    IPMZ_TRACE("capture: instantiated");
    s->graph_flags = flags;
  }
  HIP_OK(hipGraphLaunch(s->gexec, st));
  IPMZ_TRACE("graph launched");
  s->last_step_graph = 1;
  return IPMZ_OK;
}

// sticky error words of every persistent-kernel workspace the step uses
int qp_status(ipmz_qp* s) {
  hipStream_t st = s->ctx->stream;
  if (s->mixed) {
    unsigned e[2] = {0, 0};
    HIP_OK(hipMemcpyAsync(&e[0], s->mw.pctrl + PANEL_ERR_WORD, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(&e[1], s->mw.ctrl + SOLVE_ERR_WORD, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (e[0] || e[1]) return fail(IPMZ_ERR_HIP, "Newton step: a hand-off inside a persistent kernel of the "
                                                 "mixed-precision factor / solve timed out; the step is invalid");
    return IPMZ_OK;
  }
  if (s->normal) {
    const NormalWs w = normal_ws(s->nws, s->n, s->m + s->p, s->ctx);
    return ws_status(st, w.wsK, s->N, nbo_for(s->ctx, s->N), s->ctx->nbi, "Newton step (normal equations)");
  }
  if (s->B == 1 && !s->eqnone) return ws_status(st, s->ws, s->N, nbo_for(s->ctx, s->N), s->ctx->nbi, "Newton step");
  // only a step whose factor ran the two-workgroup kernel has a word to read
  // (that kernel's launch zeroes it; the default wave-specialized factor at
  // C4's N = 320 has no cross-workgroup hand-off and needs no sync here)
  if (!s->eqnone && s->ctx->nbi == 64 && small_pair_used(s->small_kernel, s->pflags != nullptr, s->B, s->N)) {
    unsigned e = 0;
    HIP_OK(hipMemcpyAsync(&e, s->pflags + (size_t)s->B * IPMZ_PAIR_FLAGS, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (e) return fail(IPMZ_ERR_HIP, "Newton step: a hand-off of the two-workgroup batched factor timed out; the "
                                     "step is invalid");
  }
  if (s->bkws) {
    unsigned e[2] = {0, 0};
    HIP_OK(hipMemcpyAsync(&e[0], bk_grid_err_word(s->bkws, s->N), 4, hipMemcpyDeviceToHost, st));
    if (s->bkfws)
      HIP_OK(hipMemcpyAsync(&e[1], bk_ws(s->bkfws, s->N).ctrl + SOLVE_ERR_WORD, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (e[0]) return fail(IPMZ_ERR_HIP, "Newton step: a grid barrier of the whole-device Bunch-Kaufman factor timed "
                                        "out; the step is invalid");
    if (e[1]) return fail(IPMZ_ERR_HIP, "Newton step: a hand-off inside the persistent triangular solve of the "
                                        "Bunch-Kaufman factor timed out; the step is invalid");
  }
  return IPMZ_OK;  // batched / one-workgroup Bunch-Kaufman kernels have no cross-workgroup spins
}

int scalars_impl(ipmz_qp* s, double* out, int count) {
  HIP_OK(hipSetDevice(s->ctx->device));
  // the B scalar blocks are one allocation with a stride: one 2-D copy
  const size_t pitch = (s->B > 1 ? (s->hq[1].scal - s->hq[0].scal) : SC_COUNT) * 8;
  HIP_OK(hipMemcpy2DAsync(out, SC_COUNT * 8, s->hq[0].scal, pitch, SC_COUNT * 8, count, hipMemcpyDeviceToHost,
                          s->ctx->stream));
  HIP_OK(hipStreamSynchronize(s->ctx->stream));
  return s->loaded ? qp_status(s) : IPMZ_OK;
}

// EqualityHandling::SlackedSlacks / NaiveSlacks: the step's slots hold [lambda_g lambda_v],
// [lambda_h lambda_w], [g v], [h w]; the reference's Newton order is
// lambda_g, lambda_h, lambda_v, lambda_w, ..., g, h, v, w (formulations.txt).
// perm[k] = the step-vector index of reference-order element k.
std::vector<int64_t> eqss_perm(const ipmz_qp* s) {
  const int64_t n = s->n, m = s->m_usr, p = s->p_usr, mp = m + p;
  const int64_t ny = s->vlo ? n : 0, nz = s->vup ? n : 0;
  std::vector<int64_t> perm;
  perm.reserve((size_t)s->state_len);
  auto run = [&](int64_t from, int64_t len) {
    for (int64_t k = 0; k < len; ++k) perm.push_back(from + k);
  };
  // x, [lambda_A lambda_C], [s t] (SlackedSlacks) or x alone (NaiveSlacks, no
  // s / lambda_A): same order
  int64_t off = s->naive ? n : n + 2 * mp;
  run(0, off);
  const int64_t LGo = off, LHo = off + mp;  // [lambda_g lambda_v], [lambda_h lambda_w]
  run(LGo, m);
  run(LHo, m);
  run(LGo + m, p);
  run(LHo + m, p);
  off += 2 * mp;
  run(off, ny + nz);  // lambda_y, lambda_z
  off += ny + nz;
  const int64_t Go = off, Ho = off + mp;  // [g v], [h w]
  run(Go, m);
  run(Ho, m);
  run(Go + m, p);
  run(Ho + m, p);
  off += 2 * mp;
  run(off, s->state_len - off);  // y, z
  return perm;
}

int get_state_impl(ipmz_qp* s, int i, int which, double* out) {
  if (which < 0 || which > 3 || !out) return fail(IPMZ_ERR_INVALID, "bad arguments");
  HIP_OK(hipSetDevice(s->ctx->device));
  const QPDev& q = s->hq[i];
  const double* src = which == 0 ? q.v[0] : which == 1 ? q.daff[0] : which == 2 ? q.dir[0] : q.r[0];
  if (s->eqss) {
    std::vector<double> tmp((size_t)s->state_len);
    HIP_OK(hipMemcpyAsync(tmp.data(), src, s->state_len * 8, hipMemcpyDeviceToHost, s->ctx->stream));
    HIP_OK(hipStreamSynchronize(s->ctx->stream));
    const auto perm = eqss_perm(s);
    for (int64_t k = 0; k < s->state_len; ++k) out[k] = tmp[(size_t)perm[(size_t)k]];
    return IPMZ_OK;
  }
  HIP_OK(hipMemcpyAsync(out, src, s->state_len * 8, hipMemcpyDeviceToHost, s->ctx->stream));
  HIP_OK(hipStreamSynchronize(s->ctx->stream));
  return IPMZ_OK;
}

// a host iterate in the reference's order -> the step's order
std::vector<double> state_in(const ipmz_qp* s, const double* in) {
  std::vector<double> v(in, in + s->state_len);
  if (s->eqss) {
    const auto perm = eqss_perm(s);
    for (int64_t k = 0; k < s->state_len; ++k) v[(size_t)perm[(size_t)k]] = in[k];
  }
  return v;
}
}  // namespace

extern "C" {

int ipmz_qp_create(ipmz_ctx* ctx, const ipmz_qp_config* cfg, ipmz_qp** out) { return create_solver(ctx, cfg, 1, out); }

int ipmz_qp_destroy(ipmz_qp* s) {
  if (!s) return IPMZ_OK;
  hipSetDevice(s->ctx->device);
  hipStreamSynchronize(s->ctx->stream);
  if (s->gexec) hipGraphExecDestroy(s->gexec);
  if (s->graph) hipGraphDestroy(s->graph);
  for (auto e : s->ev) hipEventDestroy(e);
  if (s->step_done) hipEventDestroy(s->step_done);
  if (s->step_in) hipEventDestroy(s->step_in);
  if (s->tr_pairs) {
    for (int i = 0; i < s->tr_cap; ++i) {
      hipEventDestroy(s->tr_pairs[i][0]);
      hipEventDestroy(s->tr_pairs[i][1]);
    }
    delete[] s->tr_pairs;
  }
  for (void* p : s->allocs) hipFree(p);
  if (s->mw.hev) hipEventDestroy(s->mw.hev);
  if (s->mw.hst) hipHostFree(s->mw.hst);
  ipmz_ctx* ctx = s->ctx;
  delete s;
  bool last;
  {
    std::lock_guard<std::mutex> lk(g_ctx_mutex);
    last = --ctx->users == 0 && ctx->closed;
  }
  if (last) ctx_free(ctx);
  return IPMZ_OK;
}

int ipmz_qp_load_host(ipmz_qp* s, const double* Q, const double* c, const double* A, const double* lA,
                      const double* uA, const double* C, const double* d, const double* lx, const double* ux) {
  if (!s) return fail(IPMZ_ERR_INVALID, "null qp");
  for (int i = 0; i < s->B; ++i) {
    int rc = load_one(s, i, Q, c, A, lA, uA, C, d, lx, ux);
    if (rc) return rc;
  }
  HIP_OK(qp_init_iterate(s->qb, s->ctx->stream));
  int rc = evaluate_and_save(s);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(s->ctx->stream));
  return IPMZ_OK;
}

int ipmz_qp_generate(ipmz_qp* s, uint64_t seed) {
  if (!s) return fail(IPMZ_ERR_INVALID, "null qp");
  HIP_OK(hipSetDevice(s->ctx->device));
  hipStream_t st = s->ctx->stream;
  HIP_OK(qp_generate(s->qb, seed, st));
  HIP_OK(qp_init_iterate(s->qb, st));
  int rc = evaluate_and_save(s);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(st));
  return IPMZ_OK;
}

int ipmz_qp_step(ipmz_qp* s, int flags) { return step_impl(s, flags); }

int ipmz_qp_last_step_graph(ipmz_qp* s) { return s ? s->last_step_graph : 0; }

int ipmz_qp_scalars(ipmz_qp* s, double* out) {
  if (!s || !out) return fail(IPMZ_ERR_INVALID, "null argument");
  return scalars_impl(s, out, 1);  // QP 0 (the ipmz_qp_* accessors address QP 0)
}

int ipmz_qp_device_scalars(ipmz_qp* s, double** out) {
  if (!s || !out) return fail(IPMZ_ERR_INVALID, "null argument");
  *out = s->hq[0].scal;
  return IPMZ_OK;
}

int ipmz_qp_copy_scalars(ipmz_qp* s, double* dst) {
  if (!s || !dst) return fail(IPMZ_ERR_INVALID, "null argument");
  HIP_OK(hipSetDevice(s->ctx->device));
  HIP_OK(hipMemcpyAsync(dst, s->hq[0].scal, SC_COUNT * 8, hipMemcpyDeviceToDevice, s->ctx->stream));
  return IPMZ_OK;
}

int ipmz_qp_solve(ipmz_qp* s, int max_iter, double* trace, int* iterations) {
  if (!s || !s->loaded) return fail(IPMZ_ERR_STATE, "load or generate the QP first");
  double sc[SC_COUNT];
  int rc = scalars_impl(s, sc, 1);
  if (rc) return rc;
  int it = 0;
  for (; it < max_iter; ++it) {  // Optimizer.cpp:127-135
    double* row = trace ? trace + 8 * (int64_t)it : nullptr;
    if (row) {
      row[0] = sc[SC_F];
      row[1] = sc[SC_RES];
      row[2] = sc[SC_MU];
      row[7] = sc[SC_CONVERGED];
      row[3] = row[4] = row[5] = row[6] = 0.0;
    }
    if (sc[SC_CONVERGED] != 0.0) break;
    rc = step_impl(s, 0);
    if (rc) return rc;
    rc = scalars_impl(s, sc, 1);
    if (rc) return rc;
    if (row) {
      row[3] = sc[SC_ALPHA_AFF];
      row[4] = sc[SC_MU_AFF];
      row[5] = sc[SC_SIGMA];
      row[6] = sc[SC_ALPHA];
    }
  }
  if (iterations) *iterations = it;
  return IPMZ_OK;
}

int64_t ipmz_qp_state_len(ipmz_qp* s) { return s ? s->state_len : 0; }

int ipmz_qp_get_state(ipmz_qp* s, int which, double* out) {
  if (!s) return fail(IPMZ_ERR_INVALID, "null qp");
  return get_state_impl(s, 0, which, out);
}

int ipmz_qp_set_state(ipmz_qp* s, const double* in) {
  if (!s || !in) return fail(IPMZ_ERR_INVALID, "bad arguments");
  HIP_OK(hipSetDevice(s->ctx->device));
  const std::vector<double> v = state_in(s, in);
  for (int i = 0; i < s->B; ++i)
    HIP_OK(hipMemcpyAsync(s->hq[i].v[0], v.data(), s->state_len * 8, hipMemcpyHostToDevice, s->ctx->stream));
  HIP_OK(qp_evaluate(s->qb, s->ctx->stream));
  HIP_OK(hipStreamSynchronize(s->ctx->stream));
  s->loaded = true;
  return IPMZ_OK;
}

int ipmz_qp_kkt_dim(ipmz_qp* s) { return s ? s->N : 0; }

int ipmz_qp_get_kkt(ipmz_qp* s, double* out) {
  if (!s || !out) return fail(IPMZ_ERR_INVALID, "bad arguments");
  HIP_OK(hipSetDevice(s->ctx->device));
  hipStream_t st = s->ctx->stream;
  HIP_OK(qp_assemble(s->qb, st));
  HIP_OK(hipMemcpy2DAsync(out, (size_t)s->N * 8, s->K, s->ldk * 8, (size_t)s->N * 8, s->N, hipMemcpyDeviceToHost,
                          st));
  HIP_OK(hipStreamSynchronize(st));
  for (int i = 0; i < s->N; ++i)
    for (int j = i + 1; j < s->N; ++j) out[(int64_t)i * s->N + j] = 0.0;
  return IPMZ_OK;
}

int ipmz_qp_set_mixed_precision(ipmz_qp* s, int enable, double tol, int max_refine) {
  if (!s) return fail(IPMZ_ERR_INVALID, "null qp");
  if (enable && (s->B != 1 || !(tol > 0.0) || max_refine < 0 || s->normal || s->eqnone || s->eqpen))
    return fail(IPMZ_ERR_INVALID, "mixed precision: single QPs, tol > 0, max_refine >= 0, augmented reduction, "
                                  "Regularization equalities");
  HIP_OK(hipSetDevice(s->ctx->device));
  if (enable && !s->mws) {
    const int64_t bytes = mixed_ws_bytes(s->N, nbo_for(s->ctx, s->N));
    void* w = nullptr;
    if (hipMalloc(&w, (size_t)bytes) != hipSuccess) return fail(IPMZ_ERR_NOMEM, "device allocation failed");
    s->allocs.push_back(w);
    HIP_OK(hipMemset(w, 0, (size_t)bytes));  // sticky error words start clear
    s->mws = static_cast<char*>(w);
    mixed_ws_carve(s->mws, s->N, nbo_for(s->ctx, s->N), s->mw);
    void* h = nullptr;  // the stop test's host-mapped word (eager solves wait on it)
    if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return fail(IPMZ_ERR_NOMEM, "host allocation failed");
    s->mw.hst = static_cast<unsigned*>(h);
    s->mw.hst[0] = s->mw.hst[1] = 0u;
    void* hd = nullptr;
    HIP_OK(hipHostGetDevicePointer(&hd, h, 0));
    s->mw.hst_dev = static_cast<unsigned*>(hd);
    HIP_OK(hipEventCreateWithFlags(&s->mw.hev, hipEventDisableTiming));
  }
  s->mixed = enable != 0;
  s->ir_tol = tol;
  s->ir_max = max_refine;
  if (s->gexec) {  // the captured step has the other solver baked in
    hipGraphExecDestroy(s->gexec);
    hipGraphDestroy(s->graph);
    s->gexec = nullptr;
    s->graph = nullptr;
  }
  return IPMZ_OK;
}

int ipmz_qp_set_reduction(ipmz_qp* s, int reduction) {
  if (!s) return fail(IPMZ_ERR_INVALID, "null qp");
  if (reduction != IPMZ_REDUCTION_AUGMENTED && reduction != IPMZ_REDUCTION_NORMAL)
    return fail(IPMZ_ERR_INVALID, "unknown reduction");
  if (reduction == IPMZ_REDUCTION_NORMAL && (s->B != 1 || s->mixed || s->eqnone || s->eqpen || s->naive))
    return fail(IPMZ_ERR_INVALID, "normal equations: single QPs, not with mixed precision, Regularization equalities");
  HIP_OK(hipSetDevice(s->ctx->device));
  if (reduction == IPMZ_REDUCTION_NORMAL && !s->nws) {
    const int64_t bytes = normal_ws(nullptr, s->n, s->m + s->p, s->ctx).total;
    void* w = nullptr;
    if (hipMalloc(&w, (size_t)bytes) != hipSuccess) return fail(IPMZ_ERR_NOMEM, "device allocation failed");
    s->allocs.push_back(w);
    HIP_OK(hipMemset(w, 0, (size_t)bytes));  // sticky error words start clear
    s->nws = static_cast<char*>(w);
  }
  s->normal = reduction == IPMZ_REDUCTION_NORMAL;
  if (s->gexec) {
    hipGraphExecDestroy(s->gexec);
    hipGraphDestroy(s->graph);
    s->gexec = nullptr;
    s->graph = nullptr;
  }
  return IPMZ_OK;
}

int ipmz_qp_set_timing(ipmz_qp* s, int enable) {
  if (!s) return fail(IPMZ_ERR_INVALID, "null qp");
  HIP_OK(hipSetDevice(s->ctx->device));
  s->timing = enable != 0;
  if (s->timing && s->ev.empty()) {
    s->ev.resize(8);
    for (size_t i = 0; i < s->ev.size(); ++i) HIP_OK(hipEventCreate(&s->ev[i]));
    s->tr_cap = (s->N + 63) / 64 + 8;
    s->tr_pairs = new hipEvent_t[s->tr_cap][2];
    for (int i = 0; i < s->tr_cap; ++i) {
      HIP_OK(hipEventCreate(&s->tr_pairs[i][0]));
      HIP_OK(hipEventCreate(&s->tr_pairs[i][1]));
    }
  }
  for (double& x : s->ph_ms) x = 0.0;
  s->tr_flops = 0.0;
  s->tr_launches = 0;
  return IPMZ_OK;
}

int ipmz_qp_phase_times(ipmz_qp* s, double* ms, double* flops, int64_t* launches) {
  if (!s) return fail(IPMZ_ERR_INVALID, "null qp");
  if (ms)
    for (int i = 0; i < IPMZ_PH_COUNT; ++i) ms[i] = s->ph_ms[i];
  if (flops) *flops = s->tr_flops;
  if (launches) *launches = s->tr_launches;
  return IPMZ_OK;
}

// ---- batches of independent QPs (config C4) ---------------------------------
int ipmz_batch_create(ipmz_ctx* ctx, const ipmz_qp_config* cfg, int batch, ipmz_qp** out) {
  return create_solver(ctx, cfg, batch, out);
}
int ipmz_batch_size(ipmz_qp* s) { return s ? s->B : 0; }
int ipmz_batch_load_host(ipmz_qp* s, int index, const double* Q, const double* c, const double* A, const double* lA,
                         const double* uA, const double* C, const double* d, const double* lx, const double* ux) {
  int rc = check_index(s, index);
  if (rc) return rc;
  if ((rc = load_one(s, index, Q, c, A, lA, uA, C, d, lx, ux))) return rc;
  // the kept KKT matrix K0 (off-diagonal part written only by
  // evaluate_and_save) and the residuals still hold the old data: no step
  // until ipmz_batch_initialize rebuilds them
  s->loaded = false;
  return IPMZ_OK;
}
int ipmz_batch_initialize(ipmz_qp* s) {
  if (!s) return fail(IPMZ_ERR_INVALID, "null qp");
  HIP_OK(hipSetDevice(s->ctx->device));
  HIP_OK(qp_init_iterate(s->qb, s->ctx->stream));
  int rc = evaluate_and_save(s);
  if (rc) return rc;
  HIP_OK(hipStreamSynchronize(s->ctx->stream));
  return IPMZ_OK;
}
int ipmz_batch_scalars(ipmz_qp* s, double* out) {
  if (!s || !out) return fail(IPMZ_ERR_INVALID, "null argument");
  return scalars_impl(s, out, s->B);
}
int ipmz_batch_get_state(ipmz_qp* s, int index, int which, double* out) {
  int rc = check_index(s, index);
  if (rc) return rc;
  return get_state_impl(s, index, which, out);
}
int ipmz_batch_set_state(ipmz_qp* s, int index, const double* in) {
  int rc = check_index(s, index);
  if (rc) return rc;
  if (!in) return fail(IPMZ_ERR_INVALID, "null state");
  HIP_OK(hipSetDevice(s->ctx->device));
  const std::vector<double> v = state_in(s, in);
  HIP_OK(hipMemcpyAsync(s->hq[index].v[0], v.data(), s->state_len * 8, hipMemcpyHostToDevice, s->ctx->stream));
  HIP_OK(qp_evaluate(s->qb, s->ctx->stream));
  HIP_OK(hipStreamSynchronize(s->ctx->stream));
  return IPMZ_OK;
}
int ipmz_batch_copy_scalars(ipmz_qp* s, double* dst) {
  if (!s || !dst) return fail(IPMZ_ERR_INVALID, "null argument");
  HIP_OK(hipSetDevice(s->ctx->device));
  // the B scalar blocks are one allocation with a stride of SC_COUNT doubles
  HIP_OK(hipMemcpy2DAsync(dst, SC_COUNT * 8, s->hq[0].scal, (s->B > 1 ? (s->hq[1].scal - s->hq[0].scal) : SC_COUNT) * 8,
                          SC_COUNT * 8, s->B, hipMemcpyDeviceToDevice, s->ctx->stream));
  return IPMZ_OK;
}
int ipmz_batch_summary(ipmz_qp* s, double* dst) {
  if (!s || !dst) return fail(IPMZ_ERR_INVALID, "null argument");
  HIP_OK(hipSetDevice(s->ctx->device));
  HIP_OK(qp_batch_summary(s->qb, dst, s->ctx->stream));
  return IPMZ_OK;
}
// Steps until every QP converged or max_iter; a converged QP keeps its
// iterate.  converged_count: host, may be NULL.
int ipmz_batch_solve(ipmz_qp* s, int max_iter, int* iterations, int* converged_count) {
  if (!s || !s->loaded) return fail(IPMZ_ERR_STATE, "load or generate the batch first");
  std::vector<double> sc((size_t)s->B * SC_COUNT);
  int it = 0, nconv = 0;
  for (;; ++it) {
    int rc = scalars_impl(s, sc.data(), s->B);
    if (rc) return rc;
    nconv = 0;
    for (int i = 0; i < s->B; ++i) nconv += sc[(size_t)i * SC_COUNT + SC_CONVERGED] != 0.0;
    if (nconv == s->B || it >= max_iter) break;
    if ((rc = step_impl(s, 0))) return rc;
  }
  if (iterations) *iterations = it;
  if (converged_count) *converged_count = nconv;
  return IPMZ_OK;
}
int ipmz_batch_set_factor_kernel(ipmz_qp* s, int kernel) {
  if (!s || kernel < IPMZ_BATCH_FACTOR_AUTO || kernel > IPMZ_BATCH_FACTOR_LEFT)
    return fail(IPMZ_ERR_INVALID, "ipmz_batch_set_factor_kernel: bad arguments");
  if (kernel == IPMZ_BATCH_FACTOR_PAIR && !(s->pflags && small_pair_eligible(s->B, s->N)))
    return fail(IPMZ_ERR_INVALID, "ipmz_batch_set_factor_kernel: two workgroups per QP need a batch of small systems "
                                  "(N <= 1024) with 2 * batch <= #CU");
  if (s->gexec) {  // the captured step has the other kernel baked in
    hipGraphExecDestroy(s->gexec);
    hipGraphDestroy(s->graph);
    s->gexec = nullptr;
    s->graph = nullptr;
  }
  s->small_kernel = kernel;
  return IPMZ_OK;
}

}  // extern "C"
