// Normal-equations reduction of the augmented KKT system (BASELINE config C2;
// the reference builds it symbolically, SymbolicOptimization.cpp:465-478,
// Optimizer.cpp:39-40, but never evaluates it -- SURVEY.md §0.4).
//
// With K = [[H, B^T], [B, -E]] (H = Q + Y^-1 L_y + Z^-1 L_z SPD, B = [A; C],
// E = diag((G^-1 L_g + H_h^-1 L_h)^-1, delta^2) > 0), K [x; l] = [r0; r1] is
//   S l = B H^{-1} r0 - r1,   S = E + B H^{-1} B^T   (SPD),
//   x   = H^{-1} (r0 - B^T l).
// Factor: Cholesky of H (as L D L^T with D > 0: the blocked LDL^T of
// ldlt.hip on the leading n x n block), the triangular solve
// Vt = B L^{-T} (right-looking over 128-column blocks with the solve prep's
// X_J = L_JJ^{-1}, fp64 MFMA), the
// rank-n update S = E + Vt D^{-1} Vt^T (fp64 MFMA, lower tiles only), and the
// Cholesky of S.  Solve: two solves with H, one with S, two GEMVs with B.
// B itself is left in K (the solve's GEMVs read it); Vt lives in the
// workspace.  A non-positive pivot of H or S is reported like a non-finite
// one of the LDL^T factor: 1-based index in the augmented numbering.
#include "common.h"
#include "kernels.h"

namespace ipmz {

namespace {
constexpr int NNT = 256;
}

// info <- min(index + 1) over D[i] <= 0 or non-finite (SPD check)
__global__ void k_ne_check_pos(const double* __restrict__ D, int N, int offset, int* __restrict__ info) {
  const int i = blockIdx.x * NNT + threadIdx.x;
  if (i < N && !(D[i] > 0.0 && D[i] <= 1.7976931348623157e308)) atomicMin(info, offset + i + 1);
}

// lower triangle incl. the diagonal: X <- -X   (the (2,2) block -E -> E)
__global__ __launch_bounds__(NNT) void k_ne_negate_lower(double* __restrict__ X, int64_t ld, int N) {
  const int i = blockIdx.x;
  for (int j = threadIdx.x; j <= i; j += NNT) X[(int64_t)i * ld + j] = -X[(int64_t)i * ld + j];
}

// W = -Vt D^{-1} (column scaling)
__global__ __launch_bounds__(NNT) void k_ne_scale(const double* __restrict__ Vt, int64_t ldv, int rows, int cols,
                                                  const double* __restrict__ D, double* __restrict__ W) {
  const int i = blockIdx.x;
  for (int j = threadIdx.x; j < cols; j += NNT) W[(int64_t)i * ldv + j] = -Vt[(int64_t)i * ldv + j] / D[j];
}

// t = B u - r1 : one wave per row of B
__global__ __launch_bounds__(NNT) void k_ne_gemv(const double* __restrict__ Bm, int64_t ld, int rows, int cols,
                                                 const double* __restrict__ u, const double* r1, double* t) {
  const int row = blockIdx.x * (NNT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  const double* Br = Bm + (int64_t)row * ld;
  double s = 0.0;
  for (int j = lane; j < cols; j += 64) s = fma(Br[j], u[j], s);
  s = wave_sum(s);
  if (lane == 0) t[row] = s - r1[row];
}

// partial column sums of B^T l over row chunks of 64: part[chunk][j]
__global__ __launch_bounds__(NNT) void k_ne_gemvt_part(const double* __restrict__ Bm, int64_t ld, int rows, int cols,
                                                       const double* __restrict__ l, double* __restrict__ part) {
  const int j = blockIdx.x * NNT + threadIdx.x, c = blockIdx.y;
  if (j >= cols) return;
  const int i0 = 64 * c, i1 = i0 + 64 < rows ? i0 + 64 : rows;
  double s = 0.0;
  for (int i = i0; i < i1; ++i) s = fma(Bm[(int64_t)i * ld + j], l[i], s);
  part[(int64_t)c * cols + j] = s;
}
// v = r0 - sum_chunks part (in place on r0)
__global__ void k_ne_gemvt_final(int cols, int nchunk, const double* __restrict__ part, double* __restrict__ r0) {
  const int j = blockIdx.x * NNT + threadIdx.x;
  if (j >= cols) return;
  double s = 0.0;
  for (int c = 0; c < nchunk; ++c) s += part[(int64_t)c * cols + j];
  r0[j] -= s;
}

// ---------------------------------------------------------------------------
// Launchers (the factor / solve orchestration, which reuses the LDL^T
// factor + solve entry points, is host code in capi.cpp).
hipError_t ne_check_pos(const double* D, int N, int offset, int* info, hipStream_t st) {
  if (N <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_ne_check_pos, dim3((N + NNT - 1) / NNT), dim3(NNT), 0, st, D, N, offset, info);
  return hipGetLastError();
}

// Vt <- Vt L^{-T} for the unit-lower n x n factor L (in K, ld) whose nb x nb
// diagonal-block inverses are LinvH (row-major nb x nb each, zero outside a
// partial last block): right-looking over nb-column blocks (nb <= 128)
hipError_t ne_trsm_right(double* Vt, int64_t ldv, int rows, int n, const double* K, int64_t ld, const double* LinvH,
                         int nb, hipStream_t st) {
  hipError_t e = hipSuccess;
  for (int k0 = 0; k0 < n && e == hipSuccess; k0 += nb) {
    const int bk = n - k0 < nb ? n - k0 : nb;
    // Vt[:, k] = Vt[:, k] L_kk^{-T}, in place: one tile column (BN = 128 >= nb) per row band
    e = gemm_nt_store(rows, bk, bk, Vt + k0, ldv, LinvH + (int64_t)(k0 / nb) * nb * nb, nb, Vt + k0, ldv, st);
    const int k1 = k0 + bk;
    if (e == hipSuccess && k1 < n)
      e = gemm_nt_sub_rect(rows, n - k1, bk, Vt + k0, ldv, K + (int64_t)k1 * ld + k0, ld, Vt + k1, ldv, st);
  }
  return e;
}

// -E -> E in the (2,2) block, then W = -Vt D^{-1}, then E -= W Vt^T = S
hipError_t ne_schur(double* K22, int64_t ld, int mp, const double* Vt, double* W, int64_t ldv, int n,
                    const double* DH, hipStream_t st) {
  hipLaunchKernelGGL(k_ne_negate_lower, dim3(mp), dim3(NNT), 0, st, K22, ld, mp);
  hipLaunchKernelGGL(k_ne_scale, dim3(mp), dim3(NNT), 0, st, Vt, ldv, mp, n, DH, W);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return gemm_nt_sub(mp, mp, n, W, ldv, Vt, ldv, K22, ld, 0, 0, true, st);
}

// t = B u - r1 (t may alias r1)
hipError_t ne_gemv(const double* Bm, int64_t ld, int rows, int cols, const double* u, const double* r1, double* t,
                   hipStream_t st) {
  hipLaunchKernelGGL(k_ne_gemv, dim3((rows + 3) / 4), dim3(NNT), 0, st, Bm, ld, rows, cols, u, r1, t);
  return hipGetLastError();
}

// r0 -= B^T l   (part: ceil(rows/64) * cols doubles of scratch)
hipError_t ne_gemvt(const double* Bm, int64_t ld, int rows, int cols, const double* l, double* part, double* r0,
                    hipStream_t st) {
  const int nchunk = (rows + 63) / 64;
  hipLaunchKernelGGL(k_ne_gemvt_part, dim3((cols + NNT - 1) / NNT, nchunk), dim3(NNT), 0, st, Bm, ld, rows, cols, l,
                     part);
  hipLaunchKernelGGL(k_ne_gemvt_final, dim3((cols + NNT - 1) / NNT), dim3(NNT), 0, st, cols, nchunk, part, r0);
  return hipGetLastError();
}

}  // namespace ipmz
