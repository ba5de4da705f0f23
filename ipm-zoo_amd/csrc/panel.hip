// Fused panel step: ONE launch per 64-column inner block of an outer panel,
// replacing the diag -> panel TRSM -> strip-update kernel chain of
// factor_panel (ldlt.hip).  Replaces, for that block, the column loop of
// LinearSolvers::ldlt_decomposition (LinearSolvers.cpp:20-40).
//
// Work items are tickets claimed in dependency order from a device counter
// (a ticket only waits on lower tickets, so any dispatch order is safe):
//   ticket 0      : factor the 64 x 64 diagonal block (diag64_body: L, D,
//                   L^{-1}), publish  -> flag DIAG
//   ticket 1..R   : the R <= nbo/64 - 1 row chunks inside the outer panel's
//                   diagonal region; ticket > R: the row chunks below it.
//                   Each chunk (64 rows) loads its A rows BEFORE waiting on
//                   DIAG (overlapping the diagonal factorization), then
//                     T = A L11^{-T} (MFMA), W = T, L = T / D       (TRSM)
//                   region chunks publish their W rows -> flag REG[c]; then
//                     A[rows, rest of panel] -= L W_region^T        (strip)
//                   64 columns at a time as REG flags arrive.
// The launch's ctrl words reset themselves: the last workgroup to finish
// zeroes them, so back-to-back launches (and graph replays) need no memset.
#include "common.h"
#include "diag64.h"
#include "kernels.h"
#include "sync.h"

namespace ipmz {

namespace {
enum { PC_TICKET = 0, PC_DONE = 1, PC_ERR = 2, PC_DIAG = 3, PC_REG = 4 };
constexpr int PC_WORDS = 4 + IPMZ_NBO_MAX / 64;
static_assert(PC_WORDS <= IPMZ_PANEL_CTRL_WORDS, "panel ctrl area too small");
}  // namespace

__global__ __launch_bounds__(256) void panel_step_kernel(double* __restrict__ K, int64_t ld, int N, int j0, int bi,
                                                         int c1, double* __restrict__ D, double* __restrict__ Lb,
                                                         double* __restrict__ Wc, int ldw, int* __restrict__ info,
                                                         unsigned* __restrict__ ctrl) {
  __shared__ __attribute__((aligned(16))) double smem[3 * 64 * DS + 64];
  __shared__ unsigned sh_ticket, sh_ok;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) sh_ticket = atomicAdd(&ctrl[PC_TICKET], 1u);
  __syncthreads();
  const int t = (int)sh_ticket;
  unsigned* err = &ctrl[PC_ERR];
  const int r0 = j0 + bi;              // first row below the diagonal block
  const int ce = c1 < N ? c1 : N;      // end of the outer panel's columns
  const int ncols = ce - r0;           // panel columns right of this block
  if (t == 0) {
    diag64_body<true>(K, ld, j0, bi, D, Lb, info, smem, smem + 64 * DS, smem + 2 * 64 * DS, smem + 3 * 64 * DS,
                      nullptr);
    publish(&ctrl[PC_DIAG]);
  } else {
    const int c = t - 1, row0 = r0 + 64 * c;
    const int rows = N - row0 < 64 ? N - row0 : 64;
    const bool region = row0 < ce;
    double* As = smem;            // A rows, then L rows (64 x DS)
    double* Bs = smem + 64 * DS;  // L11^{-1}, then W pieces (64 x DS)
    {
      double v[16];  // all loads in flight before the wait
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int rr = (tid >> 6) + 4 * q, cc = tid & 63;
        const int r2 = rr < rows ? rr : 0, c2 = cc < bi ? cc : 0;
        v[q] = K[(int64_t)(row0 + r2) * ld + j0 + c2];
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int rr = (tid >> 6) + 4 * q, cc = tid & 63;
        As[rr * DS + cc] = (rr < rows && cc < bi) ? v[q] : 0.0;
      }
    }
    if (wait_flag(&ctrl[PC_DIAG], err, &sh_ok)) {
#pragma unroll 4
      for (int q = 0; q < 16; ++q) {
        const int idx = tid + 256 * q;
        Bs[(idx >> 6) * DS + (idx & 63)] = ld_sc1(&Lb[idx]);
      }
      double rd[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int col = 16 * n + (lane & 15);
        rd[n] = col < bi ? 1.0 / ld_sc1(&D[j0 + col]) : 0.0;
      }
      __syncthreads();
      // ---- TRSM: wave w owns rows 16w..16w+15, all 64 columns
      const int arow = 16 * wave + (lane & 15);
      double4_t acc[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[n] = (double4_t){0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
      for (int s = 0; s < 16; ++s) {
        const int k = 4 * s + (lane >> 4);
        const double a = As[arow * DS + k];
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[n] = mfma_f64_16x16x4(a, Bs[(16 * n + (lane & 15)) * DS + k], acc[n]);
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int col = 16 * n + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = 16 * wave + (lane >> 4) + 4 * g;
          const double w = acc[n][g], l = w * rd[n];
          As[row * DS + col] = l;  // this wave's rows only
          if (row < rows && col < bi) {
            double* wp = &Wc[(int64_t)(row0 + row) * ldw + col];
            if (region) st_sc1(wp, w);
            else *wp = w;
            K[(int64_t)(row0 + row) * ld + j0 + col] = l;
          }
        }
      }
      if (region) publish(&ctrl[PC_REG + c]);
      // ---- strip: A[rows, r0 + 64q ..) -= L W_q^T, region pieces q (q <= c for region rows)
      const int npieces = ncols > 0 ? (ncols + 63) / 64 : 0;
      for (int q = 0; q < npieces; ++q) {
        if (region && q > c) break;
        if (!wait_flag(&ctrl[PC_REG + q], err, &sh_ok)) break;  // also: Bs is free
#pragma unroll 4
        for (int u = 0; u < 16; ++u) {
          const int kk = (tid >> 6) + 4 * u, cc = tid & 63;
          const int wr = r0 + 64 * q + kk;
          Bs[kk * DS + cc] = (wr < ce && cc < bi) ? ld_sc1(&Wc[(int64_t)wr * ldw + cc]) : 0.0;
        }
        __syncthreads();
        const int cbase = r0 + 64 * q;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const int cabs = cbase + 16 * n + (lane & 15);
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int row = 16 * wave + (lane >> 4) + 4 * g;
            const bool ok = row < rows && cabs < ce && cabs <= row0 + row;
            acc[n][g] = ok ? K[(int64_t)(row0 + row) * ld + cabs] : 0.0;
          }
        }
#pragma unroll 4
        for (int s = 0; s < 16; ++s) {
          const int k = 4 * s + (lane >> 4);
          const double a = -As[arow * DS + k];
#pragma unroll
          for (int n = 0; n < 4; ++n) acc[n] = mfma_f64_16x16x4(a, Bs[(16 * n + (lane & 15)) * DS + k], acc[n]);
        }
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const int cabs = cbase + 16 * n + (lane & 15);
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int row = 16 * wave + (lane >> 4) + 4 * g;
            if (row < rows && cabs < ce && cabs <= row0 + row) K[(int64_t)(row0 + row) * ld + cabs] = acc[n][g];
          }
        }
      }
    }
  }
  // ---- completion: the last workgroup out zeroes the ctrl words
  __syncthreads();
  if (tid == 0) {
    const unsigned prev = __hip_atomic_fetch_add(&ctrl[PC_DONE], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      for (int i = 0; i < PC_WORDS; ++i)
        if (i != PC_ERR) __hip_atomic_store(&ctrl[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

hipError_t panel_step(double* K, int64_t ld, int N, int j0, int bi, int c1, double* D, double* Lb, double* Wc,
                      int ldw, int* info, unsigned* ctrl, hipStream_t st) {
  if (bi <= 0 || bi > 64 || c1 - (j0 + bi) > IPMZ_NBO_MAX) return hipErrorInvalidValue;
  const int r0 = j0 + bi;
  const int nch = r0 < N ? (N - r0 + 63) / 64 : 0;
  hipLaunchKernelGGL(panel_step_kernel, dim3(1 + nch), dim3(256), 0, st, K, ld, N, j0, bi, c1, D, Lb, Wc, ldw, info,
                     ctrl);
  return hipGetLastError();
}

}  // namespace ipmz
