// Dense LDL^T factorization of the (quasi-definite) KKT matrix on gfx950.
//
// Replaces LinearSolvers::ldlt_decomposition (LinearSolvers.cpp:14-42):
// same factorization (no pivoting, Vanderbei's 1e-8 zero-pivot rule,
// :26-28), re-organised as a two-level blocked right-looking algorithm:
//
//   for each outer panel of width nbo (<= IPMZ_NBO_MAX):
//     for each inner block of width nbi (64 or 128) inside it:
//       diag   : factor the nbi x nbi diagonal block in LDS (1 workgroup),
//                also build L11^{-1} by Gauss-Jordan in the same sweep
//       panel  : T = A21 . L11^{-T} (fp64 MFMA), W21 = T, L21 = T / D1
//       strip  : update the rest of the outer panel with this inner block
//     trailing : A22 -= W21 . L21^T over the lower tiles (fp64 MFMA) -- the
//                rank-nbo update that carries ~all of the N^3/3 flops.
//
// Inside one diag block the arithmetic order equals the reference's row
// loop (sum -= (L[r][k]*L[c][k])*D[k] in k order, then / D), so a matrix that
// fits one block factors bit-identically to the reference.  Across blocks the
// MFMA accumulates a block's contributions before subtracting them, which
// changes rounding at the 1e-16 level (parity tolerance: tests/).
#include "common.h"
#include "kernels.h"

namespace ipmz {

// ---------------------------------------------------------------------------
// Diagonal block: M[r][c] holds A/L in the lower triangle (r >= c) and
// X^T = L^{-T} in the strict upper triangle (r < c); X = L^{-1} is built by
// applying the elimination steps to the identity.
template <int NB, int NT>
__global__ __launch_bounds__(NT) void ldlt_diag_kernel(double* __restrict__ K, int64_t ld, int k0, int b,
                                                       double* __restrict__ D, double* __restrict__ Linv,
                                                       int* __restrict__ info) {
  __shared__ double M[NB][NB + 1];
  __shared__ double lcol[NB];
  __shared__ double dvals[NB];
  const int tid = threadIdx.x;
  for (int idx = tid; idx < NB * NB; idx += NT) {
    const int r = idx / NB, c = idx % NB;
    double v = 0.0;
    if (r < b && c <= r) v = K[(int64_t)(k0 + r) * ld + k0 + c];
    M[r][c] = v;
  }
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6;
  constexpr int NW = NT / 64;
  for (int k = 0; k < b; ++k) {
    const double s = M[k][k];
    const double dk = s == 0.0 ? 1e-8 : s;  // LinearSolvers.cpp:28
    if (tid == 0) dvals[k] = dk;
    for (int i = k + 1 + tid; i < b; i += NT) {
      const double l = M[i][k] / dk;
      M[i][k] = l;
      lcol[i] = l;
    }
    __syncthreads();
    // columns c > k: lower rows r >= c get the rank-1 update, rows r <= k
    // (upper storage of X^T) get the Gauss-Jordan row operation.
    for (int r = wave; r < b; r += NW) {
      const double lr = r > k ? lcol[r] : 0.0;
      const double xk = r < k ? M[r][k] : 1.0;  // X[k][r]
      for (int c = k + 1 + lane; c < b; c += 64) {
        if (r >= c) {
          M[r][c] = M[r][c] - (lr * lcol[c]) * dk;
        } else if (r <= k) {
          M[r][c] = M[r][c] - lcol[c] * xk;
        }
      }
    }
    __syncthreads();
  }
  // write back L (strict lower), D, and L^{-1} (NB x NB, identity-padded)
  for (int idx = tid; idx < NB * NB; idx += NT) {
    const int r = idx / NB, c = idx % NB;
    if (r < b && c < r) K[(int64_t)(k0 + r) * ld + k0 + c] = M[r][c];
    double x;
    if (r == c) x = 1.0;
    else if (c < r && r < b) x = M[c][r];
    else x = 0.0;
    Linv[idx] = x;
  }
  for (int k = tid; k < b; k += NT) {
    const double dk = dvals[k];
    D[k0 + k] = dk;
    if (!(fabs(dk) <= 1.7976931348623157e308)) atomicMin(info, k0 + k + 1);  // first non-finite pivot
  }
}

// Inverse of the unit-lower diagonal blocks of an explicit L (one workgroup
// per block, all blocks in parallel): the solve workspace for a factor that
// was not produced by ldlt_factor (ipmz_overwriting_solve_ldlt).
template <int NB, int NT>
__global__ __launch_bounds__(NT) void linv_from_l_kernel(const double* __restrict__ L, int64_t ld, int N,
                                                         double* __restrict__ Linv) {
  __shared__ double M[NB][NB + 1];
  const int k0 = blockIdx.x * NB;
  const int b = N - k0 < NB ? N - k0 : NB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = NT / 64;
  for (int idx = tid; idx < NB * NB; idx += NT) {
    const int r = idx / NB, c = idx % NB;
    M[r][c] = (r < b && c < r) ? L[(int64_t)(k0 + r) * ld + k0 + c] : 0.0;
  }
  __syncthreads();
  for (int k = 0; k < b; ++k) {
    for (int r = wave; r <= k; r += NW) {
      const double xk = r < k ? M[r][k] : 1.0;
      for (int c = k + 1 + lane; c < b; c += 64) M[r][c] = M[r][c] - M[c][k] * xk;
    }
    __syncthreads();
  }
  double* out = Linv + (int64_t)blockIdx.x * NB * NB;
  for (int idx = tid; idx < NB * NB; idx += NT) {
    const int r = idx / NB, c = idx % NB;
    out[idx] = r == c ? 1.0 : ((c < r && r < b) ? M[c][r] : 0.0);
  }
}

hipError_t linv_from_l(const double* L, int64_t ld, int N, int nbi, double* Linv, hipStream_t st) {
  const int nblk = (N + nbi - 1) / nbi;
  if (nblk == 0) return hipSuccess;
  if (nbi == 128)
    hipLaunchKernelGGL((linv_from_l_kernel<128, 512>), dim3(nblk), dim3(512), 0, st, L, ld, N, Linv);
  else if (nbi == 64)
    hipLaunchKernelGGL((linv_from_l_kernel<64, 256>), dim3(nblk), dim3(256), 0, st, L, ld, N, Linv);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// NT GEMM tile engine on v_mfma_f64_16x16x4_f64:
//   acc[i][j] = sum_k A[i][k] * B[j][k]  (A: M x Kd, B: N x Kd, row-major)
// 256 threads = 4 waves in 2 x 2; each wave owns (BM/2) x (BN/2).
// A/B fragments (lane l): row = l & 15, k = l >> 4; C/D: col = l & 15,
// row = (l >> 4) + 4 * reg (cdna_hip_programming.md §3, f64 form).
enum { EPI_SUB = 0, EPI_PANEL = 1, EPI_STORE = 2, EPI_SUB_STRIP = 3 };

struct GemmArgs {
  int M, N, Kd;
  const double* A;
  int64_t lda;
  const double* B;
  int64_t ldb;
  double* C;
  int64_t ldc;
  // EPI_PANEL: W[i][j] = acc, C[i][j] = acc / dvec[j]
  double* W;
  int64_t ldw;
  const double* dvec;
  // lower-triangle restriction: tile skipped when row0+gi_end <= col0+gj_start
  int64_t row0, col0;
  int lower;  // 0: full rectangle, 1: skip strictly-upper tiles, 2: triangular grid (row0==col0, BM==BN)
  int ntm, ntn;
};

template <int BM, int BN, int EPI>
__global__ __launch_bounds__(256) void gemm_nt_f64_kernel(GemmArgs g) {
  constexpr int BK = 16, PAD = 18;
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
  __shared__ __attribute__((aligned(16))) double As[BM * PAD];
  __shared__ __attribute__((aligned(16))) double Bs[BN * PAD];

  int tm, tn;
  if (g.lower == 2) {
    // triangular enumeration of lower tiles: bid -> (tm >= tn)
    const int bid = blockIdx.x;
    int r = (int)((sqrt(8.0 * (double)bid + 1.0) - 1.0) * 0.5);
    while ((r + 1) * (r + 2) / 2 <= bid) ++r;
    while (r * (r + 1) / 2 > bid) --r;
    tm = r;
    tn = bid - r * (r + 1) / 2;
  } else {
    tm = blockIdx.x % g.ntm;
    tn = blockIdx.x / g.ntm;
  }
  const int i0 = tm * BM, j0 = tn * BN;
  if (g.lower == 1 && g.row0 + i0 + BM - 1 < g.col0 + j0) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  double4_t acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = (double4_t){0.0, 0.0, 0.0, 0.0};

  for (int kk = 0; kk < g.Kd; kk += BK) {
    // stage A (BM x BK) and B (BN x BK): 8 threads per row, 2 doubles each
#pragma unroll
    for (int q = 0; q < (BM * BK / 2 + 255) / 256; ++q) {
      const int ch = tid + 256 * q;
      if (ch < BM * BK / 2) {
        const int r = ch >> 3, c = (ch & 7) * 2;
        const int gi = i0 + r, gk = kk + c;
        double v0 = 0.0, v1 = 0.0;
        if (gi < g.M) {
          const double* p = g.A + (int64_t)gi * g.lda + gk;
          if (gk + 1 < g.Kd) {
            const double2 t = *reinterpret_cast<const double2*>(p);
            v0 = t.x;
            v1 = t.y;
          } else if (gk < g.Kd) {
            v0 = p[0];
          }
        }
        *reinterpret_cast<double2*>(&As[r * PAD + c]) = make_double2(v0, v1);
      }
    }
#pragma unroll
    for (int q = 0; q < (BN * BK / 2 + 255) / 256; ++q) {
      const int ch = tid + 256 * q;
      if (ch < BN * BK / 2) {
        const int r = ch >> 3, c = (ch & 7) * 2;
        const int gj = j0 + r, gk = kk + c;
        double v0 = 0.0, v1 = 0.0;
        if (gj < g.N) {
          const double* p = g.B + (int64_t)gj * g.ldb + gk;
          if (gk + 1 < g.Kd) {
            const double2 t = *reinterpret_cast<const double2*>(p);
            v0 = t.x;
            v1 = t.y;
          } else if (gk < g.Kd) {
            v0 = p[0];
          }
        }
        *reinterpret_cast<double2*>(&Bs[r * PAD + c]) = make_double2(v0, v1);
      }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < BK / 4; ++s) {
      const int k = 4 * s + (lane >> 4);
      double af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = As[(wr * WM + a * 16 + (lane & 15)) * PAD + k];
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b] = Bs[(wc * WN + b * 16 + (lane & 15)) * PAD + k];
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = mfma_f64_16x16x4(af[a], bf[b], acc[a][b]);
    }
    __syncthreads();
  }

  // epilogue
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int j = j0 + wc * WN + b * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + wr * WM + a * 16 + (lane >> 4) + 4 * r;
        if (i < g.M && j < g.N) {
          const double v = acc[a][b][r];
          double* cp = g.C + (int64_t)i * g.ldc + j;
          if (EPI == EPI_SUB || EPI == EPI_SUB_STRIP) {
            *cp = *cp - v;
          } else if (EPI == EPI_PANEL) {
            g.W[(int64_t)i * g.ldw + j] = v;
            *cp = v / g.dvec[j];
          } else {
            *cp = v;
          }
        }
      }
    }
}

template <int BM, int BN, int EPI>
static hipError_t launch_gemm(GemmArgs g, hipStream_t st) {
  g.ntm = (g.M + BM - 1) / BM;
  g.ntn = (g.N + BN - 1) / BN;
  if (g.ntm == 0 || g.ntn == 0 || g.Kd == 0) return hipSuccess;
  int64_t nblk = (int64_t)g.ntm * g.ntn;
  if (g.lower == 2) nblk = (int64_t)g.ntm * (g.ntm + 1) / 2;
  hipLaunchKernelGGL((gemm_nt_f64_kernel<BM, BN, EPI>), dim3((unsigned)nblk), dim3(256), 0, st, g);
  return hipGetLastError();
}

// C[i][j] -= sum_k A[i][k] B[j][k] over the lower part of a trailing region.
hipError_t gemm_nt_sub(int M, int N, int Kd, const double* A, int64_t lda, const double* B, int64_t ldb,
                       double* C, int64_t ldc, int64_t row0, int64_t col0, bool square_lower, hipStream_t st) {
  GemmArgs g{};
  g.M = M;
  g.N = N;
  g.Kd = Kd;
  g.A = A;
  g.lda = lda;
  g.B = B;
  g.ldb = ldb;
  g.C = C;
  g.ldc = ldc;
  g.row0 = row0;
  g.col0 = col0;
  g.lower = square_lower ? 2 : 1;
  // the trailing update (square, triangular grid) and the strip update are
  // separate instantiations so kernel traces attribute them separately
  return square_lower ? launch_gemm<128, 128, EPI_SUB>(g, st) : launch_gemm<128, 128, EPI_SUB_STRIP>(g, st);
}

hipError_t gemm_nt_store(int M, int N, int Kd, const double* A, int64_t lda, const double* B, int64_t ldb,
                         double* C, int64_t ldc, hipStream_t st) {
  GemmArgs g{};
  g.M = M;
  g.N = N;
  g.Kd = Kd;
  g.A = A;
  g.lda = lda;
  g.B = B;
  g.ldb = ldb;
  g.C = C;
  g.ldc = ldc;
  g.lower = 0;
  return launch_gemm<128, 128, EPI_STORE>(g, st);
}

// ---------------------------------------------------------------------------
hipError_t ldlt_factor(double* K, int64_t ld, int N, double* D, double* Linv, double* W, int nbo, int nbi,
                       int* info, hipStream_t st, TrailTimer* timer) {
  if (N <= 0) return hipSuccess;
  if (nbi != 64 && nbi != 128) return hipErrorInvalidValue;
  if (nbo % nbi != 0 || nbo > IPMZ_NBO_MAX) return hipErrorInvalidValue;
  hipError_t e = hipSuccess;
  for (int k0 = 0; k0 < N; k0 += nbo) {
    const int bo = N - k0 < nbo ? N - k0 : nbo;
    for (int j0 = k0; j0 < k0 + bo; j0 += nbi) {
      const int bi = k0 + bo - j0 < nbi ? k0 + bo - j0 : nbi;
      double* Lb = Linv + (int64_t)(j0 / nbi) * nbi * nbi;
      if (nbi == 128)
        hipLaunchKernelGGL((ldlt_diag_kernel<128, 512>), dim3(1), dim3(512), 0, st, K, ld, j0, bi, D, Lb, info);
      else
        hipLaunchKernelGGL((ldlt_diag_kernel<64, 256>), dim3(1), dim3(256), 0, st, K, ld, j0, bi, D, Lb, info);
      if ((e = hipGetLastError()) != hipSuccess) return e;
      const int r1 = j0 + bi;
      if (r1 >= N) continue;
      // panel: rows [r1, N), output W[:, j0-k0 ..], L21 in place
      GemmArgs g{};
      g.M = N - r1;
      g.N = bi;
      g.Kd = bi;
      g.A = K + (int64_t)r1 * ld + j0;
      g.lda = ld;
      g.B = Lb;
      g.ldb = nbi;
      g.C = K + (int64_t)r1 * ld + j0;
      g.ldc = ld;
      g.W = W + (int64_t)r1 * nbo + (j0 - k0);
      g.ldw = nbo;
      g.dvec = D + j0;
      g.lower = 0;
      e = nbi == 128 ? launch_gemm<128, 128, EPI_PANEL>(g, st) : launch_gemm<128, 64, EPI_PANEL>(g, st);
      if (e != hipSuccess) return e;
      // strip update of the remaining columns of this outer panel
      const int c1 = k0 + bo;
      if (r1 < c1) {
        e = gemm_nt_sub(N - r1, c1 - r1, bi, W + (int64_t)r1 * nbo + (j0 - k0), nbo, K + (int64_t)r1 * ld + j0,
                        ld, K + (int64_t)r1 * ld + r1, ld, r1, r1, false, st);
        if (e != hipSuccess) return e;
      }
    }
    const int t0 = k0 + bo;
    if (t0 < N) {
      hipEvent_t* ev = timer ? timer->next() : nullptr;
      if (ev) hipEventRecord(ev[0], st);
      e = gemm_nt_sub(N - t0, N - t0, bo, W + (int64_t)t0 * nbo, nbo, K + (int64_t)t0 * ld + k0, ld,
                      K + (int64_t)t0 * ld + t0, ld, t0, t0, true, st);
      if (ev) hipEventRecord(ev[1], st);
      if (timer) {
        const double R = (double)(N - t0);
        timer->flops += R * (R + 1.0) * (double)bo;  // lower triangle incl. diagonal, 2 flops per FMA
      }
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

}  // namespace ipmz
