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

__global__ __launch_bounds__(BKT) void k_bk_solve(const double* __restrict__ Lb, int64_t ld, int n, int64_t sA,
                                                  const int* __restrict__ ipivb, int64_t sP, double* __restrict__ bb,
                                                  int64_t sb) {
  __shared__ double sv[BKW];
  const double* L = Lb + blockIdx.x * sA;
  const int* ipiv = ipivb + blockIdx.x * sP;
  double* b = bb + blockIdx.x * sb;
  const int tid = threadIdx.x;
  auto l = [&](int i, int j) { return L[(int64_t)i * ld + j]; };
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
  hipLaunchKernelGGL(k_bk_solve, dim3(batch), dim3(BKT), 0, st, F, ld, n, sA, ipiv, sP, b, sb);
  return hipGetLastError();
}

}  // namespace ipmz
