// Mixed-precision Newton-direction solve (BASELINE config C5): the KKT
// matrix is symmetrically scaled (S K S, S = diag(|K_ii|^{-1/2}), so fp32
// holds it whatever the iterate -- the reference's invert(0) = sqrt(DBL_MAX)
// rule, Evaluation.cpp:267-271, alone would overflow fp32), factored ONCE in
// fp32 (ldlt_factor<float>: fp32 MFMA trailing update), and every solve
// K x = b is fp64 iterative refinement around the fp32 factor:
//
//   x = 0, r = b
//   repeat: d = S (S K S)^{-1}_{fp32} S r ;  x += d ;  r = b - K x (fp64)
//   until ||r||_inf <= tol ||b||_inf or max_refine corrections
//
// The residual uses the fp64 K (lower triangle, as assembled) in ONE pass:
// each 64 x 64 tile feeds both the row sums (K_ij x_j, j <= i) and the
// column sums of the strict lower part (K_ij x_i, i > j), the latter kept as
// per-row-block partials and reduced deterministically (no atomics).
// Convergence is decided on the device; once it holds every remaining
// refinement kernel (and the fp32 solve) returns at once, so the loop needs
// no host round trip and captures into a hipGraph.  Eagerly, a pass that
// returns at once still costs its five launches (~30 us, ~1-2 ms for the
// 20-pass limit of C5), so the eager loop enqueues as many passes as the
// previous solve needed, waits for the stop test (host-mapped word) and only
// then enqueues more -- the same kernels in the same order up to the pass
// that converged, hence the same bits as the full loop.
#include <algorithm>

#include "common.h"
#include "kernels.h"

namespace ipmz {

namespace {
constexpr int MNT = 256;
enum { ST_DONE = 0, ST_ITERS = 1 };  // unsigned state words
}  // namespace

// s_i = |K_ii|^{-1/2} (1 for a zero diagonal)
__global__ void k_mx_scale(const double* __restrict__ K, int64_t ld, int N, double* __restrict__ s) {
  const int i = blockIdx.x * MNT + threadIdx.x;
  if (i < N) {
    const double d = fabs(K[(int64_t)i * ld + i]);
    s[i] = d > 0.0 ? 1.0 / sqrt(d) : 1.0;
  }
}

// K32 = fp32(S K S), lower triangle incl. the diagonal; one block per row
__global__ __launch_bounds__(MNT) void k_mx_to_f32(const double* __restrict__ K, int64_t ld, int N,
                                                   const double* __restrict__ s, float* __restrict__ K32,
                                                   int64_t ld32) {
  const int i = blockIdx.x;
  const double si = s[i];
  const double* Kr = K + (int64_t)i * ld;
  float* Or = K32 + (int64_t)i * ld32;
  for (int j = threadIdx.x; j <= i; j += MNT) Or[j] = (float)(Kr[j] * si * s[j]);
}

// x = 0, r32 = fp32(S b), state reset
__global__ void k_mx_begin(int N, const double* __restrict__ b, const double* __restrict__ s,
                           double* __restrict__ x, float* __restrict__ r32, unsigned* __restrict__ state,
                           unsigned* __restrict__ hst) {
  const int i = blockIdx.x * MNT + threadIdx.x;
  if (i < N) {
    x[i] = 0.0;
    r32[i] = (float)(s[i] * b[i]);
  }
  if (i == 0) {
    state[ST_DONE] = 0u;
    state[ST_ITERS] = 0u;
    if (hst) hst[ST_DONE] = 0u;
  }
}

// x += S d (d = the fp32 solve's output, in r32)
__global__ void k_mx_accum(int N, const double* __restrict__ s, const float* __restrict__ d, double* __restrict__ x,
                           const unsigned* __restrict__ state) {
  if (state[ST_DONE]) return;
  const int i = blockIdx.x * MNT + threadIdx.x;
  if (i < N) x[i] += s[i] * (double)d[i];
}

// One pass over the lower triangle of K: grid (ceil(nblk/2), NSPLIT).  Block
// (w, h) takes row blocks w and nblk-1-w (equal work per block) and the h-th
// slice of their column tiles.  Thread t: column c = t & 63 of a tile, rows
// rq = 16 (t >> 6) .. +16, so every load instruction reads 64 consecutive
// doubles of one row.
//   rowp[h][i]   = sum_{j in slice, j <= i} K_ij x_j
//   colp[I][j]   = sum_{i in block I, i > j} K_ij x_i      (tile (I, j/64))
constexpr int NSPLIT = 4;
__global__ __launch_bounds__(MNT) void k_mx_symv(const double* __restrict__ K, int64_t ld, int N,
                                                 const double* __restrict__ x, double* __restrict__ colp,
                                                 double* __restrict__ rowp, int nblk,
                                                 const unsigned* __restrict__ state) {
  if (state[ST_DONE]) return;
  __shared__ double red[4][64];
  const int tid = threadIdx.x, c = tid & 63, wave = tid >> 6, rq = 16 * wave;
  const int w = blockIdx.x, h = blockIdx.y;
  for (int pass = 0; pass < 2; ++pass) {
    const int I = pass ? nblk - 1 - w : w;
    if (pass && I == w) break;
    const int r0 = 64 * I;
    const int nt = I + 1;  // column tiles 0..I
    const int jb0 = (int)((int64_t)nt * h / NSPLIT), jb1 = (int)((int64_t)nt * (h + 1) / NSPLIT);
    double xr[16], racc[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int row = r0 + rq + q;
      xr[q] = row < N ? x[row] : 0.0;
      racc[q] = 0.0;
    }
    for (int jb = jb0; jb < jb1; ++jb) {
      const int col = 64 * jb + c;
      const double xc = col < N ? x[col] : 0.0;
      double kv[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int row = r0 + rq + q;
        kv[q] = (row < N && col <= row) ? K[(int64_t)row * ld + col] : 0.0;
      }
      double cp = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        racc[q] = fma(kv[q], xc, racc[q]);
        if (r0 + rq + q > col) cp = fma(kv[q], xr[q], cp);
      }
      red[wave][c] = cp;
      __syncthreads();
      if (tid < 64 && 64 * jb + tid < N)
        colp[(int64_t)I * N + 64 * jb + tid] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const double v = wave_sum(racc[q]);
      const int row = r0 + rq + q;
      if (c == 0 && row < N) rowp[(int64_t)h * N + row] = v;
    }
  }
}

// r = b - K x ; r32 = fp32(S r) ; per-block max |r|, max |b| partials
// one workgroup per 64 columns j (lane = j): the column partials colp[I][j],
// I >= j / 64, split over the 4 waves in contiguous I ranges (the 64 columns
// share the range), summed through LDS with the row sums
__global__ __launch_bounds__(MNT) void k_mx_resid(int N, const double* __restrict__ b, const double* __restrict__ s,
                                                  const double* __restrict__ colp, const double* __restrict__ rowp,
                                                  int nblk, float* __restrict__ r32, double* __restrict__ part,
                                                  const unsigned* __restrict__ state) {
  if (state[ST_DONE]) return;
  __shared__ double sh[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int jb = blockIdx.x, j = 64 * jb + lane;
  const int cnt = nblk - jb, I0 = jb + cnt * wave / 4, I1 = jb + cnt * (wave + 1) / 4;
  double a0 = 0.0, a1 = 0.0;
  if (j < N) {
    int I = I0;
    for (; I + 1 < I1; I += 2) {
      a0 += colp[(int64_t)I * N + j];
      a1 += colp[(int64_t)(I + 1) * N + j];
    }
    if (I < I1) a0 += colp[(int64_t)I * N + j];
  }
  sh[wave][lane] = a0 + a1;
  __syncthreads();
  if (wave) return;
  double rr = 0.0, bb = 0.0;
  if (j < N) {
    double kx = 0.0;
#pragma unroll
    for (int h = 0; h < NSPLIT; ++h) kx += rowp[(int64_t)h * N + j];
    kx += (sh[0][lane] + sh[1][lane]) + (sh[2][lane] + sh[3][lane]);
    const double r = b[j] - kx;
    r32[j] = (float)(s[j] * r);
    rr = fabs(r);
    bb = fabs(b[j]);
  }
  rr = wave_max(rr);
  bb = wave_max(bb);
  if (lane == 0) {
    part[2 * blockIdx.x] = rr;
    part[2 * blockIdx.x + 1] = bb;
  }
}

// convergence test: ||r||_inf <= tol ||b||_inf ; stat = {ratio, corrections}
__global__ void k_mx_check(int nparts, const double* __restrict__ part, double tol, unsigned* __restrict__ state,
                           double* __restrict__ stat, unsigned* __restrict__ hst) {
  if (state[ST_DONE]) return;
  double rr = 0.0, bb = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 64) {
    rr = fmax(rr, part[2 * i]);
    bb = fmax(bb, part[2 * i + 1]);
  }
  rr = wave_max(rr);
  bb = wave_max(bb);
  if (threadIdx.x == 0) {
    const double ratio = bb > 0.0 ? rr / bb : rr;
    if (stat) {
      stat[0] = ratio;
      stat[1] = (double)state[ST_ITERS];
    }
    const unsigned iters = state[ST_ITERS];
    if (ratio <= tol) state[ST_DONE] = 1u;
    else state[ST_ITERS] = iters + 1u;
    if (hst) {
      hst[ST_ITERS] = iters;
      hst[ST_DONE] = ratio <= tol ? 1u : 0u;
    }
  }
}

__global__ void k_mx_finish(int N, const double* __restrict__ x, double* __restrict__ b) {
  const int i = blockIdx.x * MNT + threadIdx.x;
  if (i < N) b[i] = x[i];
}

// ---------------------------------------------------------------------------
int64_t mixed_ws_bytes(int N, int nbo) {
  MixedWs w;
  return mixed_ws_carve(nullptr, N, nbo, w);
}

int64_t mixed_ws_carve(char* base, int N, int nbo, MixedWs& w) {
  const int64_t nblk = (N + 63) / 64;
  int64_t off = 0;
  auto take = [&](int64_t bytes) {
    char* p = base ? base + off : nullptr;
    off += (bytes + 255) / 256 * 256;
    return p;
  };
  w.N = N;
  w.nbo = nbo;
  w.ld32 = (N + 63) / 64 * 64;
  w.K32 = reinterpret_cast<float*>(take((int64_t)N * w.ld32 * 4));
  w.D32 = reinterpret_cast<float*>(take((int64_t)N * 4));
  w.Linv32 = reinterpret_cast<float*>(take(nblk * 64 * 64 * 4));
  w.W32 = reinterpret_cast<float*>(take(3 * (int64_t)N * nbo * 4));
  w.y32 = reinterpret_cast<float*>(take((int64_t)N * 4));
  w.z32 = reinterpret_cast<float*>(take((int64_t)N * 4));
  w.r32 = reinterpret_cast<float*>(take((int64_t)N * 4));
  w.ctrl = reinterpret_cast<unsigned*>(take(IPMZ_SOLVE_CTRL_WORDS * 4));
  w.P32 = reinterpret_cast<float*>(take(solve_prep_elems(N) * 4));
  w.state = reinterpret_cast<unsigned*>(take(64));
  w.info = reinterpret_cast<int*>(take(64));
  w.pctrl = reinterpret_cast<unsigned*>(take(panel_ctrl_words(N, nbo) * 4));
  w.s = reinterpret_cast<double*>(take((int64_t)N * 8));
  w.x = reinterpret_cast<double*>(take((int64_t)N * 8));
  w.colp = reinterpret_cast<double*>(take(nblk * N * 8));
  w.rowp = reinterpret_cast<double*>(take((int64_t)NSPLIT * N * 8));
  w.part = reinterpret_cast<double*>(take(2 * ((N + 63) / 64) * 8));
  w.stat = reinterpret_cast<double*>(take(64));
  return off;
}

hipError_t mixed_factor(const double* K, int64_t ld, MixedWs& w, hipStream_t st, hipStream_t st2, hipStream_t st3,
                        hipEvent_t* ev,
                        int nev, TrailTimer* timer, hipStream_t st4) {
  const int N = w.N;
  if (N <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_mx_scale, dim3((N + MNT - 1) / MNT), dim3(MNT), 0, st, K, ld, N, w.s);
  hipLaunchKernelGGL(k_mx_to_f32, dim3(N), dim3(MNT), 0, st, K, ld, N, w.s, w.K32, w.ld32);
  hipError_t e = solve_reset(w.y32, w.z32, sizeof(float), N, w.ctrl, st, w.info, w.pctrl,
                             panel_ctrl_words(N, w.nbo));
  if (e != hipSuccess) return e;
  if (debug_inject_mask() & IPMZ_DEBUG_CONVERT_ONLY) return hipGetLastError();
  return ldlt_factor(w.K32, w.ld32, N, w.D32, w.Linv32, w.W32, w.nbo, 64, w.info, st, timer, st2, st3, ev, nev,
                     w.pctrl, st4);
}

hipError_t mixed_solve(const double* K, int64_t ld, MixedWs& w, double* b, double tol, int max_refine,
                       hipStream_t st) {
  const int N = w.N;
  if (N <= 0) return hipSuccess;
  const int nblk = (N + 63) / 64;
  const dim3 gv((N + MNT - 1) / MNT), bt(MNT);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  hipError_t e = hipStreamIsCapturing(st, &cs);
  if (e != hipSuccess) return e;
  const bool eager = w.hst && w.hev && cs == hipStreamCaptureStatusNone && !(debug_inject_mask() & IPMZ_DEBUG_IR_FULL);
  unsigned* hst = eager ? w.hst_dev : nullptr;
  hipLaunchKernelGGL(k_mx_begin, gv, bt, 0, st, N, b, w.s, w.x, w.r32, w.state, hst);
  const int passes = max_refine + 1;
  int it = 0, chunk = eager ? std::min(std::max(w.last_iters, 1), passes) : passes;
  while (it < passes) {
    for (const int end = std::min(passes, it + chunk); it < end; ++it) {
      e = ldlt_solve_persistent(w.K32, w.ld32, N, w.D32, w.P32, w.r32, w.y32, w.z32, w.ctrl, st,
                                it ? w.state : nullptr);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL(k_mx_accum, gv, bt, 0, st, N, w.s, w.r32, w.x, w.state);
      hipLaunchKernelGGL(k_mx_symv, dim3((nblk + 1) / 2, NSPLIT), bt, 0, st, K, ld, N, w.x, w.colp, w.rowp, nblk,
                         w.state);
      hipLaunchKernelGGL(k_mx_resid, dim3((N + 63) / 64), bt, 0, st, N, b, w.s, w.colp, w.rowp, nblk, w.r32, w.part,
                         w.state);
      hipLaunchKernelGGL(k_mx_check, dim3(1), dim3(64), 0, st, (N + 63) / 64, w.part, tol, w.state, w.stat, hst);
    }
    if (!eager || it >= passes) break;
    if ((e = hipEventRecord(w.hev, st)) != hipSuccess) return e;
    if ((e = hipEventSynchronize(w.hev)) != hipSuccess) return e;
    const volatile unsigned* h = w.hst;
    if (h[ST_DONE]) {
      w.last_iters = (int)h[ST_ITERS] + 1;
      break;
    }
    chunk = 1;
  }
  if (eager && it >= passes) w.last_iters = std::max(1, passes - 1);  // learn the count next time
  hipLaunchKernelGGL(k_mx_finish, gv, bt, 0, st, N, w.x, b);
  return hipGetLastError();
}

}  // namespace ipmz
