// Triangular solves with the LDL^T factor: x = L^{-T} D^{-1} L^{-1} b.
//
// Replaces LinearSolvers::overwriting_solve_ldlt (LinearSolvers.cpp:44-74):
// forward substitution (:56-59), diagonal scaling (:62-64), backward
// substitution with L^T (:67-73).  Blocked by the factor's inner block size
// NB; the diagonal-block solves use the L11^{-1} blocks saved by the factor
// (ldlt.hip), the off-diagonal work is a wave-per-row GEMV (forward, DPP
// reductions) or a lane-per-column GEMV (backward) over the strict lower
// triangle.  HBM/latency-bound: every step reads its NB-wide panel of L once.
//
// One launch per block step.  Workgroup 0 of step J owns the NEXT diagonal
// block: it applies step J's update to those rows first and then solves
// them (its L^{-1} block is staged into LDS while the rows update), so step
// J+1 finds its block solution ready in a side buffer.  The solve runs in
// place on b (the rows a step writes are never read by a later step).
#include "common.h"
#include "kernels.h"
#include "trsv_small.h"

namespace ipmz {

constexpr int TRSV_NT = 256;

// Stage an NB x NB row-major block into LDS (padded rows) -- coalesced.
template <int NB>
__device__ __forceinline__ void stage_block(const double* __restrict__ src, double (*dst)[NB + 1]) {
  for (int idx = threadIdx.x; idx < NB * NB; idx += TRSV_NT) dst[idx / NB][idx % NB] = src[idx];
}

// y = Linv v (transpose: y = Linv^T v) from LDS; lanes own output rows, the 4
// waves split the inner index.  Result in ys (LDS).  Caller syncs before.
template <int NB>
__device__ __forceinline__ void block_apply(const double (*Ls)[NB + 1], const double* vs, double* ys,
                                            double (*part)[NB], bool transpose) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int CH = NB / 4;
#pragma unroll
  for (int q = 0; q < NB / 64; ++q) {
    const int t = lane + 64 * q;
    double s = 0.0;
#pragma unroll 8
    for (int c = wave * CH; c < (wave + 1) * CH; ++c) s += (transpose ? Ls[c][t] : Ls[t][c]) * vs[c];
    part[wave][t] = s;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < NB; t += TRSV_NT) ys[t] = (part[0][t] + part[1][t]) + (part[2][t] + part[3][t]);
  __syncthreads();
}

// prologue: y_0 = Linv_0 b_0; b_0 <- y_0 / D_0; ybuf <- y_0
template <int NB>
__global__ __launch_bounds__(TRSV_NT) void trsv_fwd_first(const double* __restrict__ Linv,
                                                          const double* __restrict__ D, double* __restrict__ b,
                                                          double* __restrict__ ybuf, int bj) {
  __shared__ double Ls[NB][NB + 1];
  __shared__ double vs[NB], ys[NB], part[4][NB];
  stage_block<NB>(Linv, Ls);
  for (int t = threadIdx.x; t < NB; t += TRSV_NT) vs[t] = t < bj ? b[t] : 0.0;
  __syncthreads();
  block_apply<NB>(Ls, vs, ys, part, false);
  for (int t = threadIdx.x; t < bj; t += TRSV_NT) {
    ybuf[t] = ys[t];
    b[t] = ys[t] / D[t];
  }
}

// Forward row update of one workgroup: rows [r_begin, r_begin + NB) (clipped
// to r_end): b_i -= L[i, j0:j0+NB] . y_J.  Each wave owns NB/4 rows; every
// global load (L rows, b, y) is issued before the first use so the step
// pays one memory latency, then wave dot products with DPP reductions.
template <int NB>
__device__ __forceinline__ void rows_update(const double* __restrict__ K, int64_t ld, int j0, int r_begin, int r_end,
                                            const double* __restrict__ yin, double* __restrict__ b, double* ys,
                                            double* bs, double* vout) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int Q = NB / 64, RW = NB / 4;
  double lv[RW][Q];
#pragma unroll
  for (int j = 0; j < RW; ++j) {
    const int i = r_begin + wave + 4 * j;
#pragma unroll
    for (int q = 0; q < Q; ++q) lv[j][q] = i < r_end ? K[(int64_t)i * ld + j0 + lane + 64 * q] : 0.0;
  }
  for (int t = threadIdx.x; t < NB; t += TRSV_NT) {
    ys[t] = yin[t];
    const int i = r_begin + t;
    bs[t] = i < r_end ? b[i] : 0.0;
  }
  __syncthreads();
  double yl[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) yl[q] = ys[lane + 64 * q];
#pragma unroll
  for (int j = 0; j < RW; ++j) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < Q; ++q) s += lv[j][q] * yl[q];
    s = wave_sum(s);
    const int t = wave + 4 * j, i = r_begin + t;
    if (lane == 0 && i < r_end) {
      const double v = bs[t] - s;
      b[i] = v;
      if (vout) vout[t] = v;
    }
  }
}

// forward step J: rows below block J: b_i -= L[i, J] . y_J.  Workgroup 0
// owns block J+1 (rows [j1, j1+bn)) and solves it afterwards; workgroup
// w > 0 owns rows [j1 + bn + (w-1) NB, +NB).
template <int NB>
__global__ __launch_bounds__(TRSV_NT) void trsv_fwd_step(const double* __restrict__ K, int64_t ld, int N, int j0,
                                                         const double* __restrict__ LinvNext,
                                                         const double* __restrict__ D, double* __restrict__ b,
                                                         const double* __restrict__ yin, double* __restrict__ yout) {
  __shared__ double Ls[NB][NB + 1];
  __shared__ double ys[NB], bs[NB], vs[NB], yn[NB], part[4][NB];
  const int j1 = j0 + NB;
  const int bn = N - j1 < NB ? N - j1 : NB;  // size of block J+1
  if (blockIdx.x != 0) {
    const int r_begin = j1 + bn + (blockIdx.x - 1) * NB;
    rows_update<NB>(K, ld, j0, r_begin, N, yin, b, ys, bs, nullptr);
    return;
  }
  stage_block<NB>(LinvNext, Ls);  // in flight with the row loads
  for (int t = threadIdx.x; t < NB; t += TRSV_NT) vs[t] = 0.0;
  rows_update<NB>(K, ld, j0, j1, j1 + bn, yin, b, ys, bs, vs);
  __syncthreads();
  block_apply<NB>(Ls, vs, yn, part, false);
  for (int t = threadIdx.x; t < bn; t += TRSV_NT) {
    yout[t] = yn[t];
    b[j1 + t] = yn[t] / D[j1 + t];
  }
}

// backward prologue: last block: x_L = Linv_L^T z_L
template <int NB>
__global__ __launch_bounds__(TRSV_NT) void trsv_bwd_first(const double* __restrict__ Linv, double* __restrict__ b,
                                                          double* __restrict__ xbuf, int jl, int bj) {
  __shared__ double Ls[NB][NB + 1];
  __shared__ double vs[NB], xs[NB], part[4][NB];
  stage_block<NB>(Linv, Ls);
  for (int t = threadIdx.x; t < NB; t += TRSV_NT) vs[t] = t < bj ? b[jl + t] : 0.0;
  __syncthreads();
  block_apply<NB>(Ls, vs, xs, part, true);
  for (int t = threadIdx.x; t < bj; t += TRSV_NT) {
    xbuf[t] = xs[t];
    b[jl + t] = xs[t];
  }
}

// backward step J (block rows [j0, j0+bj)): z_i -= sum_r L[r][i] x_r for
// i < j0.  Each workgroup owns NB columns; its 4 waves split the rows and
// reduce through LDS.  Workgroup 0 owns block J-1 and solves it afterwards.
template <int NB>
__global__ __launch_bounds__(TRSV_NT) void trsv_bwd_step(const double* __restrict__ K, int64_t ld, int j0, int bj,
                                                         const double* __restrict__ LinvPrev,
                                                         double* __restrict__ b, const double* __restrict__ xin,
                                                         double* __restrict__ xout) {
  __shared__ double Ls[NB][NB + 1];
  __shared__ double xs[NB], part[4][NB], vs[NB], xn[NB], bs[NB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int jp = j0 - NB;  // block J-1 start (j0 is a multiple of NB, >= NB)
  if (blockIdx.x == 0) stage_block<NB>(LinvPrev, Ls);
  const int c_begin = blockIdx.x == 0 ? jp : (blockIdx.x - 1) * NB;
  // issue every load first: this wave's rows of the block-row panel, x_J, b
  constexpr int CQ = NB / 64, RW = NB / 4;
  double lv[RW][CQ];
#pragma unroll
  for (int j = 0; j < RW; ++j) {
    const int r = wave + 4 * j;
#pragma unroll
    for (int q = 0; q < CQ; ++q) lv[j][q] = r < bj ? K[(int64_t)(j0 + r) * ld + c_begin + lane + 64 * q] : 0.0;
  }
  for (int t = threadIdx.x; t < NB; t += TRSV_NT) {
    xs[t] = t < bj ? xin[t] : 0.0;
    bs[t] = b[c_begin + t];
  }
  __syncthreads();
  double s[CQ];
#pragma unroll
  for (int q = 0; q < CQ; ++q) s[q] = 0.0;
#pragma unroll
  for (int j = 0; j < RW; ++j) {
    const double xr = xs[wave + 4 * j];
#pragma unroll
    for (int q = 0; q < CQ; ++q) s[q] += lv[j][q] * xr;
  }
#pragma unroll
  for (int q = 0; q < CQ; ++q) part[wave][lane + 64 * q] = s[q];
  __syncthreads();
  for (int c = threadIdx.x; c < NB; c += TRSV_NT) {
    const double t = (part[0][c] + part[1][c]) + (part[2][c] + part[3][c]);
    const double v = bs[c] - t;
    b[c_begin + c] = v;
    vs[c] = v;
  }
  if (blockIdx.x != 0) return;
  __syncthreads();
  block_apply<NB>(Ls, vs, xn, part, true);
  for (int t = threadIdx.x; t < NB; t += TRSV_NT) {
    xout[t] = xn[t];
    b[jp + t] = xn[t];
  }
}

template <int NB>
static hipError_t ldlt_solve_nb(const double* K, int64_t ld, int N, const double* D, const double* Linv, double* b,
                                double* side, hipStream_t st) {
  const int nblk = (N + NB - 1) / NB;
  double* y0 = side;  // ping-pong block-solution buffers
  double* y1 = side + NB;
  const int64_t LB = (int64_t)NB * NB;
  const int bj0 = N < NB ? N : NB;
  hipLaunchKernelGGL((trsv_fwd_first<NB>), dim3(1), dim3(TRSV_NT), 0, st, Linv, D, b, y0, bj0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  for (int J = 0; J + 1 < nblk; ++J) {
    const int j0 = J * NB, j1 = j0 + NB;
    const int bn = N - j1 < NB ? N - j1 : NB;
    const int rest = N - j1 - bn;
    const int nwg = 1 + (rest + NB - 1) / NB;
    double* yin = (J & 1) ? y1 : y0;
    double* yout = (J & 1) ? y0 : y1;
    hipLaunchKernelGGL((trsv_fwd_step<NB>), dim3(nwg), dim3(TRSV_NT), 0, st, K, ld, N, j0, Linv + (J + 1) * LB, D,
                       b, yin, yout);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  // backward
  const int jl = (nblk - 1) * NB, bl = N - jl;
  hipLaunchKernelGGL((trsv_bwd_first<NB>), dim3(1), dim3(TRSV_NT), 0, st, Linv + (nblk - 1) * LB, b, y0, jl, bl);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  for (int J = nblk - 1, it = 0; J >= 1; --J, ++it) {
    const int j0 = J * NB;
    const int bj = N - j0 < NB ? N - j0 : NB;
    const int nwg = 1 + (j0 - NB) / NB;
    double* xin = (it & 1) ? y1 : y0;
    double* xout = (it & 1) ? y0 : y1;
    hipLaunchKernelGGL((trsv_bwd_step<NB>), dim3(nwg), dim3(TRSV_NT), 0, st, K, ld, j0, bj, Linv + (J - 1) * LB, b,
                       xin, xout);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t ldlt_solve(const double* K, int64_t ld, int N, const double* D, const double* Linv, int nbi, double* b,
                      double* side, hipStream_t st) {
  if (N <= 0) return hipSuccess;
  if (nbi == 128) return ldlt_solve_nb<128>(K, ld, N, D, Linv, b, side, st);
  if (nbi == 64) return ldlt_solve_nb<64>(K, ld, N, D, Linv, b, side, st);
  return hipErrorInvalidValue;
}


// ---------------------------------------------------------------------------
// Batched solve for many small factors (config C4, N ~ 320): one workgroup
// per QP walks its NB-row blocks itself (no inter-workgroup hand-offs):
// forward  : y_J = Linv_J b_J ; z_J = y_J / D_J ; b_i -= L[i, J] y_J (i below J)
// backward : x_J = Linv_J^T z_J ;                z_i -= L[J, i]^T x_J (i above J)
template <int NB>
__global__ __launch_bounds__(TRSV_NT) void trsv_batched_kernel(const double* __restrict__ K, int64_t ld, int N,
                                                               const double* __restrict__ D,
                                                               const double* __restrict__ Linv, double* b,
                                                               int64_t sK, int64_t sD, int64_t sL, int64_t sb) {
  __shared__ double Ls[NB][NB + 1];
  __shared__ double vs[NB], ys[NB], part[4][NB];
  const int64_t q = blockIdx.x;
  K += q * sK;
  D += q * sD;
  Linv += q * sL;
  b += q * sb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nblk = (N + NB - 1) / NB;
  for (int J = 0; J < nblk; ++J) {
    const int J0 = J * NB, bj = N - J0 < NB ? N - J0 : NB;
    stage_block<NB>(Linv + (int64_t)J * NB * NB, Ls);
    for (int t = threadIdx.x; t < NB; t += TRSV_NT) vs[t] = t < bj ? b[J0 + t] : 0.0;
    __syncthreads();
    block_apply<NB>(Ls, vs, ys, part, false);  // ends with a barrier
    for (int t = threadIdx.x; t < bj; t += TRSV_NT) b[J0 + t] = ys[t] / D[J0 + t];
    // rows below: wave per row, DPP reduction
    double yl[NB / 64];
#pragma unroll
    for (int qq = 0; qq < NB / 64; ++qq) yl[qq] = ys[lane + 64 * qq];
    for (int i = J0 + NB + wave; i < N; i += 4) {
      const double* Lr = K + (int64_t)i * ld + J0;
      double s = 0.0;
#pragma unroll
      for (int qq = 0; qq < NB / 64; ++qq) s += Lr[lane + 64 * qq] * yl[qq];
      s = wave_sum(s);
      if (lane == 0) b[i] -= s;
    }
    __syncthreads();
  }
  for (int J = nblk - 1; J >= 0; --J) {
    const int J0 = J * NB, bj = N - J0 < NB ? N - J0 : NB;
    stage_block<NB>(Linv + (int64_t)J * NB * NB, Ls);
    for (int t = threadIdx.x; t < NB; t += TRSV_NT) vs[t] = t < bj ? b[J0 + t] : 0.0;
    __syncthreads();
    block_apply<NB>(Ls, vs, ys, part, true);
    for (int t = threadIdx.x; t < bj; t += TRSV_NT) b[J0 + t] = ys[t];
    // columns above: thread per column, sum over the block's rows
    for (int c = threadIdx.x; c < J0; c += TRSV_NT) {
      double s = 0.0;
      for (int r = 0; r < bj; ++r) s += K[(int64_t)(J0 + r) * ld + c] * ys[r];
      b[c] -= s;
    }
    __syncthreads();
  }
}

// one workgroup per QP: trsv_small.h
template <int NW>
__global__ __launch_bounds__(64 * NW) void trsv_small_kernel(const double* __restrict__ K, int64_t ld, int N,
                                                             const double* __restrict__ D,
                                                             const double* __restrict__ Linv,
                                                             double* __restrict__ b, int64_t sK, int64_t sD,
                                                             int64_t sL, int64_t sb) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int64_t q = blockIdx.x;
  trsv_small_body<NW>(K + q * sK, ld, N, D + q * sD, Linv + q * sL, b + q * sb, sm);
}

hipError_t ldlt_solve_batched(const double* K, int64_t ld, int N, const double* D, const double* Linv, int nbi,
                              double* b, int B, int64_t sK, int64_t sD, int64_t sL, int64_t sb, hipStream_t st) {
  if (N <= 0 || B <= 0) return hipSuccess;
  if (nbi == 64 && N <= TRSV_SMALL_NMAX) {
    // 16 waves when the batch leaves a CU per QP, 8 when QPs share CUs
    const bool wide = B <= device_cus();
    if (ld & 1) return hipErrorInvalidValue;  // (16-byte row loads: an even leading dimension)
    const int NW = wide ? 16 : 8;
    const size_t lds = trsv_small_lds(N, NW);
    if (wide)
      hipLaunchKernelGGL((trsv_small_kernel<16>), dim3(B), dim3(64 * 16), lds, st, K, ld, N, D, Linv, b, sK, sD, sL,
                         sb);
    else
      hipLaunchKernelGGL((trsv_small_kernel<8>), dim3(B), dim3(64 * 8), lds, st, K, ld, N, D, Linv, b, sK, sD, sL,
                         sb);
  } else if (nbi == 64)
    hipLaunchKernelGGL((trsv_batched_kernel<64>), dim3(B), dim3(TRSV_NT), 0, st, K, ld, N, D, Linv, b, sK, sD, sL, sb);
  else if (nbi == 128)
    hipLaunchKernelGGL((trsv_batched_kernel<128>), dim3(B), dim3(TRSV_NT), 0, st, K, ld, N, D, Linv, b, sK, sD, sL,
                       sb);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace ipmz
