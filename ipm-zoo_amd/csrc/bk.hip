// Bunch-Kaufman symmetric indefinite factorization and solve
// (LinearSolvers::symmetric_indefinite_factorization, LinearSolvers.cpp:76-207,
// and overwriting_solve_bunch_kaufman, :209-318) -- the factor the reference
// keeps for a KKT matrix with a zero diagonal block (EqualityHandling::None,
// Optimizer.cpp:65-75), §8f row f3.
//
// One workgroup of 1024 threads per matrix (a batch of matrices = a grid of
// workgroups): the pivot choice is sequential in k, the work of a step (the
// column / row maxima, the symmetric interchange, the rank-1 or rank-2
// update of the trailing triangle) is spread over the workgroup.  Every
// element is updated with the reference's own expression and operand order
// (A[i][j] -= (r A[j][k]) A[i][k];  A[i][j] -= A[i][k] wk + A[i][k+1] wk1,
// built -ffp-contract=off), from the unscaled pivot columns staged in LDS, so
// the factor (F and ipiv) is bitwise the reference's.  The solve's forward
// sweep is element-wise too; its backward dot products are tree reductions
// (1e-16-level reordering).
//
// ipiv: >= 0 a 1x1 pivot with that interchange, < 0 (-kp, on both rows) a
// 2x2 pivot.  fix_kp = 0 keeps the reference's kp = 0 for a second all-zero
// column (LinearSolvers.cpp:111-116, the solve then divides by zero);
// fix_kp = 1 records kp = k (LAPACK's choice).
#include "common.h"
#include "kernels.h"
#include "sync.h"

namespace ipmz {

namespace {
constexpr int BKT = 1024, BKW = BKT / 64;

// (value, index) arg-max over the workgroup; ties keep the smaller index,
// values that are not > 0 (zero, NaN) never win -- the reference's strictly
// greater scan from col_max = 0
__device__ void block_argmax(double v, int idx, double* sv, int* si, double& out_v, int& out_i) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (!(v > 0.0)) {
    v = 0.0;
    idx = 0x7fffffff;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double ov = __shfl_xor(v, off);
    const int oi = __shfl_xor(idx, off);
    if (ov > v || (ov == v && oi < idx)) {
      v = ov;
      idx = oi;
    }
  }
  __syncthreads();
  if (lane == 0) {
    sv[wave] = v;
    si[wave] = idx;
  }
  __syncthreads();
  v = sv[0];
  idx = si[0];
  for (int w = 1; w < BKW; ++w)
    if (sv[w] > v || (sv[w] == v && si[w] < idx)) {
      v = sv[w];
      idx = si[w];
    }
  out_v = v;
  out_i = v > 0.0 ? idx : 0;
}

__device__ double block_sum(double v, double* sv) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) sv[wave] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < BKW; ++w) s += sv[w];
  return s;
}
}  // namespace

__global__ __launch_bounds__(BKT) void k_bk_factor(double* __restrict__ Ab, int64_t ld, int n, int64_t sA,
                                                   int* __restrict__ ipivb, int64_t sP, int* __restrict__ infob,
                                                   int fix_kp) {
  extern __shared__ double col[];  // the two pivot columns, unscaled: col[i], col[n + i]
  __shared__ double sv[BKW];
  __shared__ int si[BKW];
  __shared__ double s_r, s_wk_d11, s_wk_d22, s_wk_d21;
  double* A = Ab + blockIdx.x * sA;
  int* ipiv = ipivb + blockIdx.x * sP;
  double* c0 = col;
  double* c1 = col + n;
  const double alpha = 0x1.47e0f66afed07p-1;  // (1 + sqrt(17)) / 8, LinearSolvers.cpp:82
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  auto a = [&](int i, int j) -> double& { return A[(int64_t)i * ld + j]; };
  // ref_info: the reference's own info word, 0-based (LinearSolvers.cpp:113-116
  // sets info = k), which also decides kp -- a first zero column at k = 0
  // leaves it 0, so the NEXT zero column again takes kp = k.  info: the
  // 1-based first zero column this kernel reports (0 = none).
  int info = 0, ref_info = 0;
  for (int k = 0; k < n;) {
    // ---- pivot search (LinearSolvers.cpp:98-136)
    double cmax = 0.0;
    int imax = 0;
    {
      double v = 0.0;
      int ix = 0x7fffffff;
      for (int i = k + 1 + tid; i < n; i += BKT) {
        const double t = fabs(a(i, k));
        if (t > v) {
          v = t;
          ix = i;
        }
      }
      block_argmax(v, ix, sv, si, cmax, imax);
    }
    const double akk = fabs(a(k, k));
    int step = 1, kp = 0;
    bool zero_col = false;
    if (akk == 0.0 && cmax == 0.0) {
      zero_col = true;
      if (info == 0) info = k + 1;
      if (ref_info == 0) {
        ref_info = k;
        kp = k;
      } else if (fix_kp) {
        kp = k;
      }
    } else if (akk >= alpha * cmax) {
      kp = k;
    } else {
      double v = 0.0;
      for (int j = k + tid; j < imax; j += BKT) v = fmax(v, fabs(a(imax, j)));
      double v2 = 0.0;
      for (int i = imax + 1 + tid; i < n; i += BKT) v2 = fmax(v2, fabs(a(i, imax)));
      double r1, r2;
      int d1, d2;
      block_argmax(v, 0, sv, si, r1, d1);
      block_argmax(v2, 0, sv, si, r2, d2);
      const double rmax = r1 < r2 ? r2 : r1;  // std::max
      if (akk * rmax >= alpha * cmax * cmax) kp = k;
      else if (fabs(a(imax, imax)) >= alpha * rmax) kp = imax;
      else {
        kp = imax;
        step = 2;
      }
    }
    if (!zero_col) {
      // ---- symmetric interchange of kk and kp in the trailing lower triangle
      const int kk = k + step - 1;
      __syncthreads();
      if (kp != kk) {
        for (int i = kp + 1 + tid; i < n; i += BKT) {
          const double t = a(i, kp);
          a(i, kp) = a(i, kk);
          a(i, kk) = t;
        }
        for (int j = kk + 1 + tid; j < kp; j += BKT) {
          const double t = a(kp, j);
          a(kp, j) = a(j, kk);
          a(j, kk) = t;
        }
        if (tid == 0) {
          double t = a(kp, kp);
          a(kp, kp) = a(kk, kk);
          a(kk, kk) = t;
          if (step == 2) {
            t = a(kk, k);
            a(kk, k) = a(kp, k);
            a(kp, k) = t;
          }
        }
      }
      __syncthreads();
      // ---- stage the unscaled pivot column(s)
      for (int i = k + tid; i < n; i += BKT) {
        c0[i] = a(i, k);
        if (step == 2) c1[i] = a(i, k + 1);
      }
      if (tid == 0) {
        if (step == 1) {
          s_r = 1.0 / a(k, k);
        } else if (k < n - 1) {
          double d21 = a(k + 1, k);
          const double d11 = a(k + 1, k + 1) / d21;
          const double d22 = a(k, k) / d21;
          const double t = 1.0 / (d11 * d22 - 1.0);
          s_wk_d11 = d11;
          s_wk_d22 = d22;
          s_wk_d21 = t / d21;
        }
      }
      __syncthreads();
      if (step == 1) {
        // A[i][j] -= (r W_j) W_i, k < j <= i;  then W_j *= r
        const double r = s_r;
        for (int i = k + 1 + wave; i < n; i += BKW) {
          const double wi = c0[i];
          for (int j = k + 1 + lane; j <= i; j += 64) a(i, j) -= (r * c0[j]) * wi;
        }
        __syncthreads();
        for (int j = k + 1 + tid; j < n; j += BKT) a(j, k) = c0[j] * r;
      } else if (k < n - 1) {
        const double d11 = s_wk_d11, d22 = s_wk_d22, d21 = s_wk_d21;
        // wk_j, wk1_j from the unscaled columns (replaced in LDS after use)
        for (int i = k + 2 + wave; i < n; i += BKW) {
          const double ui = c0[i], vi = c1[i];
          for (int j = k + 2 + lane; j <= i; j += 64) {
            const double wk = d21 * (d11 * c0[j] - c1[j]);
            const double wk1 = d21 * (d22 * c1[j] - c0[j]);
            a(i, j) -= (ui * wk + vi * wk1);
          }
        }
        __syncthreads();
        for (int j = k + 2 + tid; j < n; j += BKT) {
          const double wk = d21 * (d11 * c0[j] - c1[j]);
          const double wk1 = d21 * (d22 * c1[j] - c0[j]);
          a(j, k) = wk;
          a(j, k + 1) = wk1;
        }
      }
    }
    if (tid == 0) {
      if (step == 1) ipiv[k] = kp;
      else ipiv[k] = ipiv[k + 1] = -kp;
    }
    __syncthreads();
    k += step;
  }
  if (tid == 0) infob[blockIdx.x] = info;
}

// TRANS: the factor's lower triangle as its transpose LT (row j of LT =
// column j of L, contiguous; ld = the row stride of LT): every column access of
// the sweeps is then one coalesced row instead of a cache line per element
// gate (may be null): run only when *gate != 0 (the fallback of the
// device-wide solve, bk_fast_*)
template <bool TRANS>
__global__ __launch_bounds__(BKT) void k_bk_solve(const double* __restrict__ Lb, int64_t ld, int n, int64_t sA,
                                                  const int* __restrict__ ipivb, int64_t sP, double* __restrict__ bb,
                                                  int64_t sb, const unsigned* gate) {
  if (gate && *gate == 0u) return;
  __shared__ double sv[BKW];
  const double* L = Lb + blockIdx.x * sA;
  const int* ipiv = ipivb + blockIdx.x * sP;
  double* b = bb + blockIdx.x * sb;
  const int tid = threadIdx.x;
  auto l = [&](int i, int j) { return TRANS ? L[(int64_t)j * ld + i] : L[(int64_t)i * ld + j]; };
  auto swapb = [&](int p, int q) {
    if (tid == 0) {
      const double t = b[p];
      b[p] = b[q];
      b[q] = t;
    }
    __syncthreads();
  };
  // forward: L D y = P b (LinearSolvers.cpp:229-271)
  for (int k = 0; k < n;) {
    if (ipiv[k] >= 0) {
      const int kp = ipiv[k];
      if (kp != k) swapb(k, kp);
      const double m = -b[k];
      __syncthreads();
      for (int i = k + 1 + tid; i < n; i += BKT) b[i] += l(i, k) * m;
      __syncthreads();
      if (tid == 0) b[k] /= l(k, k);
      __syncthreads();
      k += 1;
    } else {
      const int kp = -ipiv[k];
      if (kp != k + 1) swapb(k + 1, kp);
      if (k < n - 1) {
        const double m0 = -b[k];
        __syncthreads();
        for (int i = k + 2 + tid; i < n; i += BKT) b[i] += l(i, k) * m0;
        __syncthreads();
        const double m1 = -b[k + 1];
        __syncthreads();
        for (int i = k + 2 + tid; i < n; i += BKT) b[i] += l(i, k + 1) * m1;
        __syncthreads();
      }
      if (tid == 0) {
        const double d21 = l(k + 1, k);
        const double d11 = l(k, k) / d21;
        const double d22 = l(k + 1, k + 1) / d21;
        const double den = d11 * d22 - 1.0;
        const double b1 = b[k] / d21, b2 = b[k + 1] / d21;
        b[k] = (d22 * b1 - b2) / den;
        b[k + 1] = (d11 * b2 - b1) / den;
      }
      __syncthreads();
      k += 2;
    }
  }
  // backward: L^T x = y, then undo the interchanges (LinearSolvers.cpp:273-317)
  auto dot_update = [&](int from, int j) {
    double s = 0.0;
    for (int i = from + tid; i < n; i += BKT) s = fma(l(i, j), b[i], s);
    s = block_sum(s, sv);
    if (tid == 0) b[j] -= s;
    __syncthreads();
  };
  for (int k = n - 1; k >= 0;) {
    if (ipiv[k] >= 0) {
      if (k < n - 1) dot_update(k + 1, k);
      const int kp = ipiv[k];
      if (kp != k) swapb(k, kp);
      k -= 1;
    } else {
      if (k < n - 1) {
        // both dot products read b[k+1..n), written by neither
        double s0 = 0.0, s1 = 0.0;
        for (int i = k + 1 + tid; i < n; i += BKT) {
          s0 = fma(l(i, k), b[i], s0);
          s1 = fma(l(i, k - 1), b[i], s1);
        }
        s0 = block_sum(s0, sv);
        __syncthreads();
        s1 = block_sum(s1, sv);
        if (tid == 0) {
          b[k] -= s0;
          b[k - 1] -= s1;
        }
        __syncthreads();
      }
      const int kp = -ipiv[k];
      if (kp != k) swapb(k, kp);
      k -= 2;
    }
  }
}

// ---------------------------------------------------------------------------
// The same factorization over the whole device (one matrix, N beyond one
// workgroup's reach -- EqualityHandling::None at headline size).
//
// The pivot choice is sequential in k and the trailing update of step k is
// all of the work, HBM-bound (the reference's right-looking rank-1 / rank-2
// update touches the trailing triangle once per step, (N-k)^2/2 elements
// read and written).  G workgroups (one per CU) stay resident for the whole
// factor and meet at a grid barrier once per step (twice when the row search
// runs).  Ownership is fixed: row i belongs to workgroup i mod G and, inside
// it, column j to thread j mod 1024, so every element of the matrix is only
// ever touched by one thread -- the bulk update needs no cross-XCD coherence
// at all.  What crosses workgroups goes through small write-through buffers:
//   * the next two pivot columns, staged by their owning threads during the
//     update (colbuf, two parities), with each workgroup's (max, argmax) of
//     the next pivot column (so the column search costs no extra pass);
//   * the row search's row i_max and column i_max (prow, pcol) with their
//     per-workgroup maxima;
// and the symmetric interchange is never applied as a pass of its own: the
// pivot columns after the interchange are read through the swap map from
// those buffers, and each owner rewrites the few interchanged elements of its
// own rows while updating them.  Arithmetic is element by element the
// reference's (same expressions, same operand order, -ffp-contract=off), so
// F and ipiv are bitwise those of LinearSolvers.cpp:76-207, as for the
// one-workgroup kernel above.
namespace bkg {
constexpr int T = 1024;  // threads per workgroup: column j -> thread j mod T
static_assert(T == BKT, "block_argmax reduces over BKT threads");

struct Layout {
  int64_t ctrl, colbuf, cpv, cpi, rp1, rp2, prow, pcol, total;
};
IPMZ_HOST_DEVICE Layout layout(int n, int G) {
  Layout l;
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    const int64_t at = o;
    o += (bytes + 255) / 256 * 256;
    return at;
  };
  l.ctrl = take(256);
  l.colbuf = take(4 * (int64_t)n * 8);  // [parity][2 columns][n]
  l.cpv = take(2 * (int64_t)G * 8);
  l.cpi = take(2 * (int64_t)G * 4);
  l.rp1 = take((int64_t)G * 8);
  l.rp2 = take((int64_t)G * 8);
  l.prow = take((int64_t)n * 8);
  l.pcol = take((int64_t)n * 8);
  l.total = o;
  return l;
}

// One pass: mode 0 stages columns lo, lo+1 only; mode 1 / 2 is the update
// of a 1x1 / 2x2 pivot at column k (lo = k + mode), with the interchange of
// rows / columns kk = lo - 1 and kp when swap.
struct Pass {
  int mode, k, lo, kp;  // mode 3: two 1x1 pivots k, k+1 without interchange in one pass (lo = k + 2)
  bool swap;
  double r, d11, d22, d21;
  double r1, s01, d1;  // mode 3: 1 / a'(k+1,k+1), r a(k+1,k), a'(k+1,k+1) (a' = after step k)
  const double *ck0, *ck1, *prow, *pcol;  // staged pre-interchange columns k, k+1; row / column i_max
  double *nb0, *nb1;                      // staging out: columns lo, lo+1
  double* cpv;                            // this workgroup's (max, argmax) slot of column lo
  int* cpi;
};
// the pivot columns AFTER the interchange (LinearSolvers.cpp:137-164 applied
// to the staged pre-interchange data)
__device__ __forceinline__ double c0v(const Pass& P, int i) {
  if (P.mode == 1) {
    if (!P.swap) return ld_sc1(P.ck0 + i);
    if (i == P.k) return ld_sc1(P.prow + P.kp);  // a(kp, kp)
    if (i < P.kp) return ld_sc1(P.prow + i);     // a(kp, i)
    if (i == P.kp) return ld_sc1(P.prow + P.k);  // a(kp, k) stays
    return ld_sc1(P.pcol + i);                   // a(i, kp)
  }
  if (P.swap && i == P.k + 1) return ld_sc1(P.prow + P.k);  // a(kk, k) <-> a(kp, k)
  if (P.swap && i == P.kp) return ld_sc1(P.ck0 + P.k + 1);
  return ld_sc1(P.ck0 + i);
}
__device__ __forceinline__ double c1v(const Pass& P, int i) {  // mode 2, i >= k + 1
  if (!P.swap) return ld_sc1(P.ck1 + i);
  if (i == P.k + 1) return ld_sc1(P.prow + P.kp);
  if (i < P.kp) return ld_sc1(P.prow + i);
  if (i == P.kp) return ld_sc1(P.prow + P.k + 1);  // a(kp, kk) stays
  return ld_sc1(P.pcol + i);
}

__device__ void pass(double* __restrict__ A, int64_t ld, int n, const Pass& P, double* rc0, double* rc1,
                     double* rsub, int g, int G, int nq) {
  const int tid = threadIdx.x, lo = P.lo;
  const int q_lo = lo <= g ? 0 : (lo - g + G - 1) / G;  // first owned row >= lo
  if (P.mode) {
    const double* ckS = P.mode == 1 ? P.ck0 : P.ck1;
    for (int q = q_lo + tid; q < nq; q += T) {
      const int i = g + q * G;
      rc0[q] = c0v(P, i);
      if (P.mode == 2) rc1[q] = c1v(P, i);
      if (P.mode == 3) rc1[q] = ld_sc1(P.ck1 + i) - P.s01 * rc0[q];  // a(i,k+1) after step k
      if (P.swap && i > P.kp) rsub[q] = ld_sc1(ckS + i);  // a(i, kp) <- a(i, kk)
    }
  }
  __syncthreads();
  if (P.mode) {
    // the interchanged elements outside the update range, and the L column(s)
    // (LinearSolvers.cpp:176-178, 199-202) -- by the owners of column k, k+1
    const int k = P.k;
    if (tid == (k & (T - 1))) {
      if (P.mode == 1 && P.swap && k % G == g) A[(int64_t)k * ld + k] = ld_sc1(P.prow + P.kp);
      if (P.mode == 2 && P.swap && (k + 1) % G == g) A[(int64_t)(k + 1) * ld + k] = ld_sc1(P.prow + k);
      if (P.mode == 3 && (k + 1) % G == g) A[(int64_t)(k + 1) * ld + k] = ld_sc1(P.ck0 + k + 1) * P.r;
      for (int q = q_lo; q < nq; ++q) {
        const int i = g + q * G;
        A[(int64_t)i * ld + k] = P.mode != 2 ? rc0[q] * P.r : P.d21 * (P.d11 * rc0[q] - rc1[q]);
      }
    }
    if (P.mode == 3 && tid == ((k + 1) & (T - 1))) {  // step k+1's pivot and L column
      if ((k + 1) % G == g) A[(int64_t)(k + 1) * ld + k + 1] = P.d1;
      for (int q = q_lo; q < nq; ++q) {
        const int i = g + q * G;
        A[(int64_t)i * ld + k + 1] = rc1[q] * P.r1;
      }
    }
    if (P.mode == 2 && tid == ((k + 1) & (T - 1))) {
      if (P.swap && (k + 1) % G == g) A[(int64_t)(k + 1) * ld + k + 1] = ld_sc1(P.prow + P.kp);
      for (int q = q_lo; q < nq; ++q) {
        const int i = g + q * G;
        A[(int64_t)i * ld + k + 1] = P.d21 * (P.d22 * rc1[q] - rc0[q]);
      }
    }
  }
  const bool kprow = P.swap && P.kp % G == g;
  double mx = 0.0;
  int mi = 0x7fffffff;
  for (int j = lo + (((tid - lo) % T) + T) % T; j < n; j += T) {
    if (!P.mode && j > lo + 1) break;
    double w0 = 0.0, w1 = 0.0, subj = 0.0;
    if (P.mode == 1) {
      w0 = P.r * c0v(P, j);
    } else if (P.mode == 3) {
      const double a0 = ld_sc1(P.ck0 + j);
      w0 = P.r * a0;
      w1 = P.r1 * (ld_sc1(P.ck1 + j) - P.s01 * a0);  // r1 a'(j,k+1)
    } else if (P.mode == 2) {
      const double a0 = c0v(P, j), a1 = c1v(P, j);
      w0 = P.d21 * (P.d11 * a0 - a1);
      w1 = P.d21 * (P.d22 * a1 - a0);
    }
    if (kprow && j <= P.kp) subj = ld_sc1((P.mode == 1 ? P.ck0 : P.ck1) + (j < P.kp ? j : lo - 1));
    const bool stage0 = j == lo, stage1 = j == lo + 1;
    int q = j <= g ? 0 : (j - g + G - 1) / G;
    // rows in groups of 4: the loads of a group are in flight together
    for (; q < nq; q += 4) {
      double v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = g + (q + u) * G;
        v[u] = q + u < nq ? A[(int64_t)i * ld + j] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (q + u >= nq) break;
        const int i = g + (q + u) * G;
        double x = v[u];
        if (P.swap) {
          if (i == P.kp && j <= P.kp) x = subj;
          else if (i > P.kp && j == P.kp) x = rsub[q + u];
        }
        if (P.mode == 1) x = x - w0 * rc0[q + u];  // a(i,j) -= (r a(j,k)) a(i,k)
        else if (P.mode == 3) {                     // step k, then step k+1 on the updated values
          x = x - w0 * rc0[q + u];
          x = x - w1 * rc1[q + u];
        } else if (P.mode == 2) x = x - (rc0[q + u] * w0 + rc1[q + u] * w1);
        if (P.mode) A[(int64_t)i * ld + j] = x;
        if (stage0) {
          st_sc1(P.nb0 + i, x);
          const double t = fabs(x);
          if (i > lo && t > mx) {  // strictly greater, rows ascending: the first maximum
            mx = t;
            mi = i;
          }
        } else if (stage1) {
          st_sc1(P.nb1 + i, x);
        }
      }
    }
  }
  if (lo < n && tid == (lo & (T - 1))) {
    st_sc1(P.cpv, mx);
    st_sc1(P.cpi, mi);
  }
}

// grid barrier: every wave drains its stores, one arrival per workgroup on a
// monotonic counter, wait for target = (barrier number) x G.  A spin past
// SPIN_TICKS (or another workgroup's) raises the sticky error word.
__device__ __forceinline__ bool gbar(unsigned* cnt, unsigned* err, unsigned target, unsigned* s_ok) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned ok = 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned it = 0; ld_sc1(cnt) < target; ++it) {
      if ((it & 255u) == 255u &&
          (ld_sc1(err) != 0u || __builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS)) {
        st_sc1(err, 1u);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0;
}

__device__ double block_fmax(double v, double* sv) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) sv[wave] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < BKW; ++w) s = fmax(s, sv[w]);
  return s;
}
}  // namespace bkg

__global__ __launch_bounds__(bkg::T) void k_bk_grid(double* __restrict__ A, int64_t ld, int n,
                                                     int* __restrict__ ipiv, int* __restrict__ infop, int fix_kp,
                                                     char* __restrict__ ws) {
  using namespace bkg;
  extern __shared__ double rows[];  // rc0, rc1, rsub of the owned rows
  __shared__ double sv[BKW];
  __shared__ int si[BKW];
  __shared__ unsigned s_ok;
  const int G = gridDim.x, g = blockIdx.x, tid = threadIdx.x;
  const Layout L = layout(n, G);
  unsigned* ctrl = reinterpret_cast<unsigned*>(ws + L.ctrl);
  double* colbuf = reinterpret_cast<double*>(ws + L.colbuf);
  double* cpv = reinterpret_cast<double*>(ws + L.cpv);
  int* cpi = reinterpret_cast<int*>(ws + L.cpi);
  double* rp1 = reinterpret_cast<double*>(ws + L.rp1);
  double* rp2 = reinterpret_cast<double*>(ws + L.rp2);
  double* prow = reinterpret_cast<double*>(ws + L.prow);
  double* pcol = reinterpret_cast<double*>(ws + L.pcol);
  const int nq = g < n ? (n - g + G - 1) / G : 0;
  double *rc0 = rows, *rc1 = rows + nq, *rsub = rows + 2 * nq;
  const double alpha = 0x1.47e0f66afed07p-1;  // (1 + sqrt(17)) / 8, LinearSolvers.cpp:82
  unsigned nbar = 0;
  int par = 0;  // parity of the last staging pass
  auto run = [&](Pass P) -> bool {
    const int out = par ^ 1;
    P.nb0 = colbuf + (2 * out) * (int64_t)n;
    P.nb1 = colbuf + (2 * out + 1) * (int64_t)n;
    P.cpv = cpv + out * G + g;
    P.cpi = cpi + out * G + g;
    pass(A, ld, n, P, rc0, rc1, rsub, g, G, nq);
    par = out;
    return gbar(ctrl, ctrl + 1, (++nbar) * (unsigned)G, &s_ok);
  };
  auto stage = [&](int lo) {
    Pass P{};
    P.mode = 0;
    P.lo = lo;
    return run(P);
  };
  int info = 0, ref_info = 0;
  bool ok = stage(0);
  for (int k = 0; ok && k < n;) {
    const double* ck0 = colbuf + (2 * par) * (int64_t)n;
    const double* ck1 = colbuf + (2 * par + 1) * (int64_t)n;
    // ---- column search from the per-workgroup maxima (LinearSolvers.cpp:104-107)
    double cmax = 0.0;
    int imax = 0;
    {
      double v = 0.0;
      int ix = 0x7fffffff;
      if (tid < G) {
        v = ld_sc1(cpv + par * G + tid);
        ix = ld_sc1(cpi + par * G + tid);
      }
      block_argmax(v, ix, sv, si, cmax, imax);
    }
    const double akk = fabs(ld_sc1(ck0 + k));
    int step = 1, kp = 0;
    bool zero_col = false;
    if (akk == 0.0 && cmax == 0.0) {
      zero_col = true;
      if (info == 0) info = k + 1;
      if (ref_info == 0) {
        ref_info = k;
        kp = k;
      } else if (fix_kp) {
        kp = k;
      }
    } else if (akk >= alpha * cmax) {
      kp = k;
    } else {
      // ---- row search (LinearSolvers.cpp:121-134): row i_max left of the
      // diagonal (its owner) and column i_max below it (every owner), each
      // published for the interchange
      double r1 = 0.0, r2 = 0.0;
      if (imax % G == g)
        for (int j = k + (((tid - k) % T) + T) % T; j <= imax; j += T) {
          const double x = A[(int64_t)imax * ld + j];
          st_sc1(prow + j, x);
          if (j < imax) r1 = fmax(r1, fabs(x));
        }
      if (tid == (imax & (T - 1))) {
        const int q0 = imax < g ? 0 : (imax - g) / G + 1;  // owned rows > imax
        for (int q = q0; q < nq; ++q) {
          const int i = g + q * G;
          const double x = A[(int64_t)i * ld + imax];
          st_sc1(pcol + i, x);
          r2 = fmax(r2, fabs(x));
        }
      }
      r1 = block_fmax(r1, sv);
      r2 = block_fmax(r2, sv);
      if (tid == 0) {
        st_sc1(rp1 + g, r1);
        st_sc1(rp2 + g, r2);
      }
      ok = gbar(ctrl, ctrl + 1, (++nbar) * (unsigned)G, &s_ok);
      if (!ok) break;
      r1 = block_fmax(tid < G ? ld_sc1(rp1 + tid) : 0.0, sv);
      r2 = block_fmax(tid < G ? ld_sc1(rp2 + tid) : 0.0, sv);
      const double rmax = r1 < r2 ? r2 : r1;  // std::max
      if (akk * rmax >= alpha * cmax * cmax) kp = k;
      else if (fabs(ld_sc1(prow + imax)) >= alpha * rmax) kp = imax;
      else {
        kp = imax;
        step = 2;
      }
    }
    // ---- pivot k+1 from the staged columns: when step k is a 1x1 pivot
    // without interchange, column k+1 after step k is ck1 - (r a(k+1,k)) ck0
    // (the reference's own update expression), so its column search and
    // pivot test need no pass; if it is a 1x1 pivot without interchange too,
    // both updates run in ONE pass (each element updated by step k, then by
    // step k+1 -- the reference's order), halving the trailing traffic.
    bool pair = false;
    double r0 = 0.0, s01 = 0.0, d1 = 0.0;
    if (!zero_col && step == 1 && kp == k && k + 1 < n) {
      r0 = 1.0 / ld_sc1(ck0 + k);
      s01 = r0 * ld_sc1(ck0 + k + 1);
      double v = 0.0, cmax1 = 0.0;
      int ix = 0x7fffffff, imax1 = 0;
      for (int i = k + 2 + tid; i < n; i += T) {
        const double t = fabs(ld_sc1(ck1 + i) - s01 * ld_sc1(ck0 + i));
        if (t > v) {
          v = t;
          ix = i;
        }
      }
      block_argmax(v, ix, sv, si, cmax1, imax1);
      d1 = ld_sc1(ck1 + k + 1) - s01 * ld_sc1(ck0 + k + 1);
      const double akk1 = fabs(d1);
      pair = !(akk1 == 0.0 && cmax1 == 0.0) && akk1 >= alpha * cmax1;
    }
    if (g == 0 && tid == 0) {
      if (step == 1) ipiv[k] = kp;
      else ipiv[k] = ipiv[k + 1] = -kp;
      if (pair) ipiv[k + 1] = k + 1;
    }
    if (pair) {
      Pass P{};
      P.mode = 3;
      P.k = k;
      P.lo = k + 2;
      P.kp = k;
      P.ck0 = ck0;
      P.ck1 = ck1;
      P.r = r0;
      P.s01 = s01;
      P.d1 = d1;
      P.r1 = 1.0 / d1;
      ok = run(P);
      k += 2;
      continue;
    }
    if (zero_col) {  // no interchange, no update: stage the next column
      if (k + 1 < n) ok = stage(k + 1);
      k += 1;
      continue;
    }
    Pass P{};
    P.mode = step;
    P.k = k;
    P.lo = k + step;
    P.kp = kp;
    P.swap = kp != k + step - 1;
    P.ck0 = ck0;
    P.ck1 = ck1;
    P.prow = prow;
    P.pcol = pcol;
    if (step == 1) {
      P.r = 1.0 / c0v(P, k);
    } else {
      const double d21 = c0v(P, k + 1);
      const double d11 = c1v(P, k + 1) / d21;
      const double d22 = c0v(P, k) / d21;
      const double t = 1.0 / (d11 * d22 - 1.0);
      P.d11 = d11;
      P.d22 = d22;
      P.d21 = t / d21;
    }
    ok = run(P);
    k += step;
  }
  if (g == 0 && tid == 0) *infop = info;
}

size_t bk_grid_ws_bytes(int n) { return (size_t)bkg::layout(n, device_cus()).total; }

hipError_t bk_factor_grid(double* A, int64_t ld, int n, int* ipiv, int* info, int fix_kp, void* ws,
                          hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int G = device_cus();
  const int nq = (n + G - 1) / G;
  // one workgroup per CU, all resident at once (a grid barrier per pivot
  // step): refuse a launch whose LDS or registers would not allow it rather
  // than let the barriers time out
  const size_t lds = 3 * (size_t)nq * sizeof(double);
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_bk_grid, bkg::T, lds) != hipSuccess || per_cu < 1)
    return hipErrorInvalidConfiguration;
  char* w = static_cast<char*>(ws);
  hipError_t e = hipMemsetAsync(w + bkg::layout(n, G).ctrl, 0, 256, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_bk_grid, dim3(G), dim3(bkg::T), lds, st, A, ld, n, ipiv, info, fix_kp, w);
  return hipGetLastError();
}

const unsigned* bk_grid_err_word(const void* ws, int n) {
  return reinterpret_cast<const unsigned*>(static_cast<const char*>(ws) + bkg::layout(n, device_cus()).ctrl) + 1;
}

hipError_t bk_factor(double* A, int64_t ld, int n, int* ipiv, int* info, int fix_kp, int batch, int64_t sA,
                     int64_t sP, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (n > IPMZ_BK_NMAX) return hipErrorInvalidValue;
  const size_t lds = 2 * (size_t)n * sizeof(double);  // <= 64 KB
  hipLaunchKernelGGL(k_bk_factor, dim3(batch), dim3(BKT), lds, st, A, ld, n, sA, ipiv, sP, info, fix_kp);
  return hipGetLastError();
}

hipError_t bk_solve(const double* F, int64_t ld, int n, const int* ipiv, double* b, int batch, int64_t sA, int64_t sP,
                    int64_t sb, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_bk_solve<false>, dim3(batch), dim3(BKT), 0, st, F, ld, n, sA, ipiv, sP, b, sb, nullptr);
  return hipGetLastError();
}

// LT[j][i] = F[i][j], i >= j (64 x 64 tiles through LDS: coalesced both ways)
__global__ __launch_bounds__(256) void k_bk_transpose(const double* __restrict__ F, int64_t ld, int n,
                                                      double* __restrict__ LT, int64_t ldt) {
  __shared__ double t[64][65];
  const int bi = blockIdx.y, bj = blockIdx.x;  // source tile rows 64 bi.., columns 64 bj..
  if (bj > bi) return;
  const int c = threadIdx.x & 63;
  for (int r = threadIdx.x >> 6; r < 64; r += 4) {
    const int i = 64 * bi + r, j = 64 * bj + c;
    t[r][c] = (i < n && j < n) ? F[(int64_t)i * ld + j] : 0.0;
  }
  __syncthreads();
  for (int r = threadIdx.x >> 6; r < 64; r += 4) {
    const int j = 64 * bj + r, i = 64 * bi + c;  // LT row j, column i
    if (j < n && i < n && i >= j) LT[(int64_t)j * ldt + i] = t[c][r];
  }
}

hipError_t bk_transpose(const double* F, int64_t ld, int n, double* LT, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int nb = (n + 63) / 64;
  hipLaunchKernelGGL(k_bk_transpose, dim3(nb, nb), dim3(256), 0, st, F, ld, n, LT, (int64_t)n);
  return hipGetLastError();
}
hipError_t bk_solve_lt(const double* LT, int n, const int* ipiv, double* b, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_bk_solve<true>, dim3(1), dim3(BKT), 0, st, LT, (int64_t)n, n, 0, ipiv, 0, b, 0, nullptr);
  return hipGetLastError();
}


// ---------------------------------------------------------------------------
// Device-wide solve (bk_fast_*).  The reference's sweeps interleave the
// interchanges with the column updates (LinearSolvers.cpp:229-317); every
// interchange of step j moves entries at positions >= j only, so it commutes
// with the updates of the columns before it once those columns' rows are
// permuted the same way.  Folding every later interchange into each column
// of L once per factor gives A^{-1} b = P^T L'^{-T} D^{-1} L'^{-1} P b with
// L' unit lower (a 2x2 pivot's d21 entry zeroed: the reference never
// updates b[k+1] from column k), D block diagonal (1x1, 2x2 as the
// reference solves them) and P the composite interchange -- so both sweeps
// are the persistent 128-row triangular solve of the LDL^T path
// (trsv_persist.hip) and the interchanges two gathers.  Falls back to the
// one-workgroup sweeps (gated by meta's flag) when an all-zero column made
// the factor singular (the reference's kp = 0 defect swaps backwards) or the
// interchange bookkeeping does not fit one workgroup's LDS.
namespace bkf {
constexpr int LDS_MAX_N = 16384;     // perm + slot map in LDS: 8 n bytes
constexpr int SLOT_MAX = 16384;      // touched positions of the interchanges (LDS doubles)
struct Meta {
  unsigned* flag;  // [0] 1 = fall back; [1] swaps; [2] slots
  int *kind, *perm, *srow, *sa, *sb, *slotpos;
  double *d11, *d21, *d22, *ones, *t;
  size_t total;
};
inline Meta layout(char* base, int n) {
  Meta m;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += (bytes + 255) / 256 * 256;
    return p;
  };
  m.flag = reinterpret_cast<unsigned*>(take(256));
  m.kind = reinterpret_cast<int*>(take((size_t)n * 4));
  m.perm = reinterpret_cast<int*>(take((size_t)n * 4));
  m.srow = reinterpret_cast<int*>(take((size_t)n * 4));
  m.sa = reinterpret_cast<int*>(take((size_t)n * 4));
  m.sb = reinterpret_cast<int*>(take((size_t)n * 4));
  m.slotpos = reinterpret_cast<int*>(take((size_t)2 * n * 4));
  m.d11 = reinterpret_cast<double*>(take((size_t)n * 8));
  m.d21 = reinterpret_cast<double*>(take((size_t)n * 8));
  m.d22 = reinterpret_cast<double*>(take((size_t)n * 8));
  m.ones = reinterpret_cast<double*>(take((size_t)n * 8));
  m.t = reinterpret_cast<double*>(take((size_t)n * 8));
  m.total = off;
  return m;
}

// One workgroup: the pivot structure in the reference's order.  kind[k]: 0
// = 1x1, 1 / 2 = first / second row of a 2x2; the interchanges in step order
// (row srow, positions sa = srow and sb = kp, as slot indices into slotpos,
// the distinct positions they touch); perm = the composite interchange
// ((P b)[p] = b[perm[p]]).  Thread 0 walks ipiv in chunks staged in LDS.
__global__ __launch_bounds__(1024) void k_scan(const int* __restrict__ ipiv, int n, const int* __restrict__ info,
                                               Meta m) {
  extern __shared__ int lds[];  // perm[n], slotof[n]
  __shared__ int chunk[1025];
  __shared__ int sh_bad, sh_ns, sh_nsl;
  int* perm = lds;
  int* slotof = lds + n;
  const int tid = threadIdx.x;
  for (int i = tid; i < n; i += 1024) {
    perm[i] = i;
    slotof[i] = -1;
  }
  if (tid == 0) {
    sh_bad = (info && *info != 0) ? 1 : 0;  // an all-zero column: the reference divides by zero
    sh_ns = 0;
    sh_nsl = 0;
  }
  __syncthreads();
  int k = 0;  // next pivot step (thread 0's; the chunk loop is uniform)
  for (int c0 = 0; c0 < n; c0 += 1024) {
    if (c0 + tid < n) chunk[tid] = ipiv[c0 + tid];
    if (tid == 0) chunk[1024] = c0 + 1024 < n ? ipiv[c0 + 1024] : 0;
    __syncthreads();
    if (tid == 0) {
      int ns = sh_ns, nsl = sh_nsl, bad = sh_bad;
      auto slot = [&](int pos) {
        if (slotof[pos] < 0) {
          if (nsl < SLOT_MAX) m.slotpos[nsl] = pos;
          slotof[pos] = nsl++;
        }
        return slotof[pos];
      };
      while (k < n && k < c0 + 1024) {
        const int p = chunk[k - c0];
        int r, kp, step;
        if (p >= 0) {
          r = k;
          kp = p;
          step = 1;
          m.kind[k] = 0;
        } else {
          r = k + 1;
          kp = -p;
          step = 2;
          m.kind[k] = 1;
          if (k + 1 < n) m.kind[k + 1] = 2;
        }
        if (kp != r && r < n) {
          if (kp < r || kp >= n) bad = 1;  // a backward interchange (the kp = 0 defect)
          else {
            m.srow[ns] = r;
            m.sa[ns] = slot(r);
            m.sb[ns] = slot(kp);
            ++ns;
            const int t = perm[r];
            perm[r] = perm[kp];
            perm[kp] = t;
          }
        }
        k += step;
      }
      sh_ns = ns;
      sh_nsl = nsl;
      sh_bad = bad || nsl > SLOT_MAX;
    }
    __syncthreads();
  }
  for (int i = tid; i < n; i += 1024) m.perm[i] = perm[i];
  if (tid == 0) {
    m.flag[0] = sh_bad ? 1u : 0u;
    m.flag[1] = (unsigned)sh_ns;
    m.flag[2] = (unsigned)sh_nsl;
  }
}

// the pivot blocks of D (from F, before it is overwritten) and the ones vector
__global__ void k_extract(const double* __restrict__ F, int64_t ld, int n, Meta m) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  m.ones[k] = 1.0;
  const double d11 = F[(int64_t)k * ld + k];
  m.d11[k] = d11;
  const int kd = m.kind[k];
  if (kd == 1) {
    m.d21[k] = F[(int64_t)(k + 1) * ld + k];
    m.d22[k] = F[(int64_t)(k + 1) * ld + k + 1];
  }
  // a zero pivot (an all-zero column): the reference divides by zero in its
  // own order -- the fallback reproduces that order
  if ((kd == 0 && d11 == 0.0) || (kd == 1 && m.d21[k] == 0.0)) atomicOr(&m.flag[0], 1u);
}

// column c of L (row c of LT): every interchange after the column's pivot
// step applied to its entries (through the touched slots, in LDS), and a 2x2
// pivot's d21 zeroed
__global__ __launch_bounds__(256) void k_lprime(double* __restrict__ LT, int n, Meta m) {
  if (m.flag[0]) return;
  extern __shared__ double vals[];
  __shared__ int sh_s0;
  const int c = blockIdx.x, tid = threadIdx.x;
  const int kd = m.kind[c];
  const int cp = kd == 1 ? c + 1 : c;  // last row of the column's pivot step
  const int ns = (int)m.flag[1], nsl = (int)m.flag[2];
  double* row = LT + (int64_t)c * n;
  if (kd == 1 && tid == 0) row[c + 1] = 0.0;
  if (tid == 0) {  // first interchange of a later step: srow > cp (srow increases)
    int lo = 0, hi = ns;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (m.srow[mid] > cp) hi = mid;
      else lo = mid + 1;
    }
    sh_s0 = lo;
  }
  __syncthreads();
  const int s0 = sh_s0;
  if (s0 >= ns) return;
  for (int t = tid; t < nsl; t += 256) {
    const int pos = m.slotpos[t];
    vals[t] = pos > cp ? row[pos] : 0.0;
  }
  __syncthreads();
  if (tid == 0)
    for (int s = s0; s < ns; ++s) {
      const int a = m.sa[s], b = m.sb[s];
      const double v = vals[a];
      vals[a] = vals[b];
      vals[b] = v;
    }
  __syncthreads();
  for (int t = tid; t < nsl; t += 256) {
    const int pos = m.slotpos[t];
    if (pos > cp) row[pos] = vals[t];
  }
}

// Lp[i][j] = LT[j][i], i > j (64 x 64 tiles through LDS)
__global__ __launch_bounds__(256) void k_untranspose(const double* __restrict__ LT, int n, double* __restrict__ Lp,
                                                     int64_t ld, const unsigned* __restrict__ flag) {
  if (flag[0]) return;
  __shared__ double t[64][65];
  const int bi = blockIdx.y, bj = blockIdx.x;  // destination tile rows 64 bi.., columns 64 bj..
  if (bj > bi) return;
  const int c = threadIdx.x & 63;
  for (int r = threadIdx.x >> 6; r < 64; r += 4) {  // LT rows 64 bj + r, columns 64 bi + c
    const int j = 64 * bj + r, i = 64 * bi + c;
    t[r][c] = (i < n && j < n && i > j) ? LT[(int64_t)j * n + i] : 0.0;
  }
  __syncthreads();
  for (int r = threadIdx.x >> 6; r < 64; r += 4) {
    const int i = 64 * bi + r, j = 64 * bj + c;
    if (i < n && j < n && i > j) Lp[(int64_t)i * ld + j] = t[c][r];
  }
}

__global__ void k_set_fallback(unsigned* flag) {
  if (threadIdx.x == 0) flag[0] = 1u;
}
__global__ void k_gather(const double* __restrict__ b, int n, Meta m) {
  if (m.flag[0]) return;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) m.t[p] = b[m.perm[p]];
}
__global__ void k_scatter(double* __restrict__ b, int n, Meta m) {
  if (m.flag[0]) return;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < n) b[m.perm[p]] = m.t[p];
}
// y <- D^{-1} y in the reference's arithmetic (LinearSolvers.cpp:238, :250-258)
__global__ void k_dsolve(double* __restrict__ y, int n, Meta m) {
  if (m.flag[0]) return;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int kd = m.kind[k];
  if (kd == 0) {
    y[k] = y[k] / m.d11[k];
  } else if (kd == 1) {
    const double akm1k = m.d21[k];
    const double akm1 = m.d11[k] / akm1k;
    const double ak = m.d22[k] / akm1k;
    const double denom = akm1 * ak - 1.0;
    const double bkm1 = y[k] / akm1k;
    const double bk = y[k + 1] / akm1k;
    y[k] = (ak * bkm1 - bk) / denom;
    y[k + 1] = (akm1 * bk - bkm1) / denom;
  }
}
}  // namespace bkf

size_t bk_fast_meta_bytes(int n) { return bkf::layout(nullptr, n).total; }
const unsigned* bk_fast_flag(const void* meta) { return static_cast<const unsigned*>(meta); }
const double* bk_fast_ones(const void* meta, int n) { return bkf::layout(static_cast<char*>(const_cast<void*>(meta)), n).ones; }
double* bk_fast_tmp(void* meta, int n) { return bkf::layout(static_cast<char*>(meta), n).t; }

hipError_t bk_fast_prepare(const double* F, int64_t ld, int n, const int* ipiv, const int* info, double* LT,
                           double* Lp, int64_t ldp, void* meta, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  bkf::Meta m = bkf::layout(static_cast<char*>(meta), n);
  if (n > bkf::LDS_MAX_N) {  // the interchange bookkeeping lives in one workgroup's LDS: fall back
    hipLaunchKernelGGL(bkf::k_set_fallback, dim3(1), dim3(64), 0, st, m.flag);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(bkf::k_scan, dim3(1), dim3(1024), (size_t)2 * n * sizeof(int), st, ipiv, n, info, m);
  hipLaunchKernelGGL(bkf::k_extract, dim3((n + 255) / 256), dim3(256), 0, st, F, ld, n, m);
  hipLaunchKernelGGL(bkf::k_lprime, dim3(n), dim3(256), (size_t)bkf::SLOT_MAX * sizeof(double), st, LT, n, m);
  const int nb = (n + 63) / 64;
  hipLaunchKernelGGL(bkf::k_untranspose, dim3(nb, nb), dim3(256), 0, st, (const double*)LT, n, Lp, ldp,
                     (const unsigned*)m.flag);
  return hipGetLastError();
}

hipError_t bk_fast_gather(const double* b, int n, void* meta, hipStream_t st) {
  hipLaunchKernelGGL(bkf::k_gather, dim3((n + 255) / 256), dim3(256), 0, st, b, n,
                     bkf::layout(static_cast<char*>(meta), n));
  return hipGetLastError();
}
hipError_t bk_fast_dsolve(double* y, int n, void* meta, hipStream_t st) {
  hipLaunchKernelGGL(bkf::k_dsolve, dim3((n + 255) / 256), dim3(256), 0, st, y, n,
                     bkf::layout(static_cast<char*>(meta), n));
  return hipGetLastError();
}
hipError_t bk_fast_scatter(double* b, int n, void* meta, hipStream_t st) {
  hipLaunchKernelGGL(bkf::k_scatter, dim3((n + 255) / 256), dim3(256), 0, st, b, n,
                     bkf::layout(static_cast<char*>(meta), n));
  return hipGetLastError();
}
hipError_t bk_fast_fallback(const double* LT, int n, const int* ipiv, double* b, const void* meta, hipStream_t st) {
  hipLaunchKernelGGL(k_bk_solve<true>, dim3(1), dim3(BKT), 0, st, LT, (int64_t)n, n, 0, ipiv, 0, b, 0,
                     bk_fast_flag(meta));
  return hipGetLastError();
}

}  // namespace ipmz
