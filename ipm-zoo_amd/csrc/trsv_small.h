// The small-factor batched solve's per-QP body (trsv.hip trsv_small_kernel,
// and newton.hip k_fused_solves, which runs it twice per Newton step with the
// fused middle phases in between).  Included by both; one workgroup of NW
// waves per QP, sm: trsv_small_lds(N, NW) bytes of LDS.
#pragma once
#include "common.h"

namespace ipmz {

constexpr int TRSV_SMALL_NMAX = 4096;  // trsv_small_body: 2 N doubles of LDS (kernels.h fused_solves_ok)
__host__ __device__ constexpr size_t trsv_small_lds(int N, int NW) {
  return (2 * (size_t)((N + 63) & ~63) + 2 * NW * 64 + 64) * sizeof(double);
}

// Small-factor batched solve (config C4, N <= TRSV_SMALL_NMAX, NB = 64):
// one workgroup of NW waves per QP, the whole vector in LDS and both sweeps
// LEFT-looking, so every block step is ONE round of independent, coalesced
// global loads (no read-modify-write of b in global memory, no serial
// per-row chains):
//   forward : u_J = b_J - L[J, 0:J0] y[0:J0]      (row segments, lanes over
//             columns, waves over the block's rows, DPP row sums)
//             y_J = Linv_J u_J
//   scale   : z = y / D
//   backward: u_J = z_J - L[J0+64:N, J]^T x[J0+64:N] (64-wide row segments,
//             lane = column, waves over rows, LDS cross-wave sum)
//             x_J = Linv_J^T u_J
// Linv_J is read from global memory (row-major, identity-padded) with its
// loads issued ahead of the step's dot products.
template <int NW>
__device__ __forceinline__ void trsv_small_body(const double* __restrict__ K, int64_t ld, int N,
                                                const double* __restrict__ D, const double* __restrict__ Linv,
                                                double* __restrict__ b, double* __restrict__ sm) {
  constexpr int RW = 64 / NW;  // block rows per wave
  const int Np = (N + 63) & ~63;
  double* bv = sm;                 // rhs, then x
  double* yv = sm + Np;            // y, then z
  // K is read 16 bytes per lane in the backward sweep (two rows per
  // instruction) and, in the 16-wave kernel (a CU per QP), the forward one:
  // B = 128 solve 0.070 -> 0.068 ms, B = 1024 0.334 -> 0.332 ms; the 8-wave
  // forward sweep was slower so (0.344 ms; profiles/r04_race/solve16_*)
  constexpr bool W16 = NW >= 16;
  double* part = yv + Np;          // 2 NW x 64 partial sums
  double* ub = part + 2 * NW * 64; // 64: the block's u
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int t = tid; t < Np; t += 64 * NW) {
    bv[t] = t < N ? b[t] : 0.0;
    yv[t] = 0.0;
  }
  __syncthreads();
  const int nblk = Np / 64;
  // ---- forward
  for (int J = 0; J < nblk; ++J) {
    const int J0 = 64 * J, bj = N - J0 < 64 ? N - J0 : 64;
    const double* Lb = Linv + (int64_t)J * 64 * 64;
    double lv[RW], acc[RW];
#pragma unroll
    for (int k = 0; k < RW; ++k) {
      // (the strict upper triangle of Linv_J is zero: not loaded, 62.5 % of
      // the block's 128-byte lines fetched)
      lv[k] = lane <= wave * RW + k ? Lb[(wave * RW + k) * 64 + lane] : 0.0;
      acc[k] = 0.0;
    }
    // (W16) 128-column chunks as 16-byte loads (lane: columns c0 + 2 lane,
    // + 1), then 64-column ones
    int c0 = 0;
#pragma unroll 2
    for (; W16 && c0 + 128 <= J0; c0 += 128) {
      const double2 yc = *reinterpret_cast<const double2*>(&yv[c0 + 2 * lane]);
#pragma unroll
      for (int k = 0; k < RW; ++k) {
        const int r = wave * RW + k;
        const int rr = r < bj ? r : 0;  // clamp: rows past N read row J0 (discarded)
        const double2 kv = *reinterpret_cast<const double2*>(&K[(int64_t)(J0 + rr) * ld + c0 + 2 * lane]);
        acc[k] = fma(kv.x, yc.x, acc[k]);
        acc[k] = fma(kv.y, yc.y, acc[k]);
      }
    }
#pragma unroll 2
    for (; c0 < J0; c0 += 64) {
      const double yc = yv[c0 + lane];
#pragma unroll
      for (int k = 0; k < RW; ++k) {
        const int r = wave * RW + k;
        const int rr = r < bj ? r : 0;  // clamp: rows past N read row J0 (discarded)
        acc[k] = fma(K[(int64_t)(J0 + rr) * ld + c0 + lane], yc, acc[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < RW; ++k) {
      const double s = wave_sum(acc[k]);
      const int r = wave * RW + k;
      if (lane == 0) ub[r] = r < bj ? bv[J0 + r] - s : 0.0;
    }
    __syncthreads();
    const double uc = ub[lane];
#pragma unroll
    for (int k = 0; k < RW; ++k) {
      const double s = wave_sum(lv[k] * uc);
      const int r = wave * RW + k;
      if (lane == 0 && r < bj) yv[J0 + r] = s;
    }
    __syncthreads();
  }
  // ---- z = y / D
  for (int t = tid; t < N; t += 64 * NW) yv[t] = yv[t] / D[t];
  __syncthreads();
  // ---- backward
  for (int J = nblk - 1; J >= 0; --J) {
    const int J0 = 64 * J, bj = N - J0 < 64 ? N - J0 : 64;
    const double* Lb = Linv + (int64_t)J * 64 * 64;
    double lv[RW];
#pragma unroll
    for (int k = 0; k < RW; ++k) lv[k] = lane <= wave * RW + k ? Lb[(wave * RW + k) * 64 + lane] : 0.0;
    // two rows per load instruction: half-wave h takes rows i = J0 + 64 +
    // 2 wave + h (+ 2 NW), lane l & 31 columns 2 (l & 31), + 1 (16 bytes)
    const int h = lane >> 5, c2 = 2 * (lane & 31);
    double2 acc = {0.0, 0.0};
#pragma unroll 4
    for (int i = J0 + 64 + 2 * wave + h; i < N; i += 2 * NW) {
      const double2 kv = *reinterpret_cast<const double2*>(&K[(int64_t)i * ld + J0 + c2]);
      const double xb = bv[i];
      acc.x = fma(kv.x, xb, acc.x);
      acc.y = fma(kv.y, xb, acc.y);
    }
    part[(2 * wave + h) * 64 + c2] = acc.x;
    part[(2 * wave + h) * 64 + c2 + 1] = acc.y;
    __syncthreads();
    if (wave == 0) {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < 2 * NW; ++w) s += part[w * 64 + lane];
      ub[lane] = lane < bj ? yv[J0 + lane] - s : 0.0;
    }
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < RW; ++k) t = fma(lv[k], ub[wave * RW + k], t);
    part[wave * 64 + lane] = t;
    __syncthreads();
    if (wave == 0 && lane < bj) {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += part[w * 64 + lane];
      bv[J0 + lane] = s;
    }
    __syncthreads();
  }
  for (int t = tid; t < N; t += 64 * NW) b[t] = bv[t];
}

}  // namespace ipmz
