// The whole outer panel of the blocked LDL^T in ONE launch: replaces, for
// nbo columns, the column loop of LinearSolvers::ldlt_decomposition
// (LinearSolvers.cpp:20-40).  Inner 64-column blocks hand off to each other
// by flags inside the launch instead of kernel boundaries.
#include "common.h"
#include "diag64.h"
#include "kernels.h"
#include "sync.h"

namespace ipmz {

// ---------------------------------------------------------------------------
// The whole outer panel in ONE launch.  Columns [k0, c1), c1 = k0 + bo, as
// nb = ceil(bo/64) inner blocks j; rows [k0, N) as 64-row chunks c, one
// workgroup each (ticket = chunk, so a chunk only ever waits on lower
// tickets).  Chunk c walks the blocks j = 0 .. min(c, nb-1) in order:
//   c == j (region chunk on the diagonal): factor the 64 x 64 block,
//          publish DIAG[j]; done.
//   c >  j: T = A[c, j] L_jj^{-T} (waits DIAG[j]); L[c, j] = T / D_j;
//          W[c, j] = T; region chunks publish REG[j][c];
//          strip: A[c, q] -= L[c, j] W[q, j]^T for q = j+1 .. min(c, nb-1)
//          (waits REG[j][q]).
// The chain between two diagonal factorizations is one 64-row TRSM and one
// 64 x 64 strip piece of the next region chunk, instead of a kernel boundary
// behind ALL rows of the previous inner block (panel_step_kernel).
// Data written earlier in the same launch is read with agent-scope loads.
namespace {
enum { OP_TICKET = 0, OP_DONE = 1, OP_ERR = PANEL_ERR_WORD, OP_DIAG = 4, OP_REG = 16 };
constexpr int OP_NBMAX = IPMZ_NBO_MAX / 64;
constexpr int OP_WORDS = OP_REG + OP_NBMAX * OP_NBMAX;
static_assert(OP_DIAG + OP_NBMAX <= OP_REG, "ctrl layout");
static_assert(OP_WORDS <= IPMZ_PANEL_CTRL_WORDS, "panel ctrl area too small");
}  // namespace

// T = float: the fp32 factor of the mixed-precision path (f32 MFMA TRSM and
// strip pieces; the diagonal block is factored in fp64 and stored in fp32).
template <typename T>
__global__ __launch_bounds__(256) void outer_panel_kernel(T* __restrict__ K, int64_t ld, int N, int k0, int c1,
                                                          T* __restrict__ D, T* __restrict__ Lb0, T* __restrict__ Wp,
                                                          int ldw, int* __restrict__ info,
                                                          unsigned* __restrict__ ctrl, int inject) {
  typedef Mfma<T> MF;
  typedef typename MF::acc_t acc_t;
  __shared__ __attribute__((aligned(16))) double smem[2 * 64 * DS + 64];
  __shared__ unsigned sh_ticket, sh_ok;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) sh_ticket = atomicAdd(&ctrl[OP_TICKET], 1u);
  __syncthreads();
  const int c = (int)sh_ticket;
  unsigned* err = &ctrl[OP_ERR];
  const int ce = c1 < N ? c1 : N;  // end of the panel's columns
  const int nb = (ce - k0 + 63) / 64;
  const int row0 = k0 + 64 * c;
  const int rows = N - row0 < 64 ? N - row0 : 64;
  const bool region = c < nb;
  const int jend = region ? c : nb;  // blocks this chunk TRSMs: j < jend
  T* As = reinterpret_cast<T*>(smem);              // A rows, then L rows (64 x DS)
  T* Bs = reinterpret_cast<T*>(smem + 64 * DS);  // L_jj^{-1}, then W pieces (64 x DS)
  const int arow = 16 * wave + (lane & 15);
  bool ok = true;
  for (int j = 0; j < jend && ok; ++j) {
    const int j0 = k0 + 64 * j;
    const int bj = ce - j0 < 64 ? ce - j0 : 64;
    T* Lb = Lb0 + (int64_t)j * 64 * 64;
    {  // this chunk's A rows of block j: loads in flight before the wait
      T v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int rr = (tid >> 6) + 4 * q, cc = tid & 63;
        const int r2 = rr < rows ? rr : 0, c2 = cc < bj ? cc : 0;
        const T* src = &K[(int64_t)(row0 + r2) * ld + j0 + c2];
        v[q] = j ? ld_sc1(src) : *src;
      }
      __syncthreads();  // previous block's strip finished reading As / Bs
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int rr = (tid >> 6) + 4 * q, cc = tid & 63;
        As[rr * DS + cc] = (rr < rows && cc < bj) ? v[q] : T(0);
      }
    }
    if (!(ok = wait_flag(&ctrl[OP_DIAG + j], err, &sh_ok))) break;
#pragma unroll 4
    for (int q = 0; q < 16; ++q) {
      const int idx = tid + 256 * q;
      Bs[(idx >> 6) * DS + (idx & 63)] = ld_sc1(&Lb[idx]);
    }
    T rd[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = 16 * n + (lane & 15);
      rd[n] = col < bj ? T(1) / ld_sc1(&D[j0 + col]) : T(0);
    }
    // region chunk: its own diagonal block (columns of block c), the target
    // of this iteration's first strip piece -- loads in flight during the TRSM
    acc_t own[4];
    if (region) {
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int cabs = row0 + 16 * n + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = 16 * wave + MF::row(lane, g);
          const bool in = row < rows && cabs < ce && cabs <= row0 + row;
          const T* src = &K[(int64_t)(row0 + (in ? row : 0)) * ld + (in ? cabs : k0)];
          own[n][g] = in ? (j ? ld_sc1(src) : *src) : T(0);
        }
      }
    }
    __syncthreads();
    // ---- TRSM: wave w owns rows 16w..16w+15, all 64 columns
    acc_t acc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[n] = (acc_t){T(0), T(0), T(0), T(0)};
#pragma unroll 4
    for (int s = 0; s < 16; ++s) {
      const int k = 4 * s + (lane >> 4);
      const T a = As[arow * DS + k];
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[n] = MF::mma(a, Bs[(16 * n + (lane & 15)) * DS + k], acc[n]);
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = 16 * n + (lane & 15);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int row = 16 * wave + MF::row(lane, g);
        const T w = acc[n][g], l = w * rd[n];
        As[row * DS + col] = l;  // this wave's rows only
        if (row < rows && col < bj) {
          T* wp = &Wp[(int64_t)(row0 + row) * ldw + 64 * j + col];
          if (region) st_sc1(wp, w);
          else *wp = w;
          K[(int64_t)(row0 + row) * ld + j0 + col] = l;
        }
      }
    }
    if (region) {
      publish(&ctrl[OP_REG + j * OP_NBMAX + c]);  // (its barrier also frees Bs)
      // ---- own piece first: A[c, c] -= L[c, j] W[c, j]^T with W from this
      // workgroup's registers through LDS, no global round trip -- for
      // j = c - 1 it is the last link of the chain to this chunk's diagonal
      // factorization
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int col = 16 * n + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) Bs[(16 * wave + MF::row(lane, g)) * DS + col] = acc[n][g];
      }
      __syncthreads();
#pragma unroll 4
      for (int s = 0; s < 16; ++s) {
        const int k = 4 * s + (lane >> 4);
        const T a = -As[arow * DS + k];
#pragma unroll
        for (int n = 0; n < 4; ++n) own[n] = MF::mma(a, Bs[(16 * n + (lane & 15)) * DS + k], own[n]);
      }
      if (j + 1 < c) {  // more blocks to come: back to K (re-read with sc1)
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const int cabs = row0 + 16 * n + (lane & 15);
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int row = 16 * wave + MF::row(lane, g);
            if (row < rows && cabs < ce && cabs <= row0 + row) K[(int64_t)(row0 + row) * ld + cabs] = own[n][g];
          }
        }
      } else {  // final: straight into the diagonal factorization's LDS image
        const int bc = ce - row0 < 64 ? ce - row0 : 64;
        double* M = smem;
        __syncthreads();  // every wave done reading As / Bs
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const int col = 16 * n + (lane & 15);
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int row = 16 * wave + MF::row(lane, g);
            M[row * DS + col] = (row < bc && col <= row) ? (double)own[n][g] : (row == col ? 1.0 : 0.0);
          }
        }
      }
    }
    // ---- strip: A[c, q] -= L[c, j] W[q, j]^T, q = j+1 .. (region: c - 1; else nb-1)
    const int qend = region ? c - 1 : nb - 1;
    for (int q = j + 1; q <= qend; ++q) {
      if (!(ok = wait_flag(&ctrl[OP_REG + j * OP_NBMAX + q], err, &sh_ok))) break;  // also: Bs is free
      const int cbase = k0 + 64 * q;
#pragma unroll 4
      for (int u = 0; u < 16; ++u) {
        const int kk = (tid >> 6) + 4 * u, cc = tid & 63;
        const int wr = cbase + kk;
        Bs[kk * DS + cc] = (wr < ce && cc < bj) ? ld_sc1(&Wp[(int64_t)wr * ldw + 64 * j + cc]) : T(0);
      }
      __syncthreads();
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int cabs = cbase + 16 * n + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = 16 * wave + MF::row(lane, g);
          const bool in = row < rows && cabs < ce && cabs <= row0 + row;
          const T* src = &K[(int64_t)(row0 + (in ? row : 0)) * ld + (in ? cabs : k0)];
          acc[n][g] = in ? (j ? ld_sc1(src) : *src) : T(0);
        }
      }
#pragma unroll 4
      for (int s = 0; s < 16; ++s) {
        const int k = 4 * s + (lane >> 4);
        const T a = -As[arow * DS + k];
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[n] = MF::mma(a, Bs[(16 * n + (lane & 15)) * DS + k], acc[n]);
      }
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int cabs = cbase + 16 * n + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = 16 * wave + MF::row(lane, g);
          if (row < rows && cabs < ce && cabs <= row0 + row) K[(int64_t)(row0 + row) * ld + cabs] = acc[n][g];
        }
      }
      __syncthreads();  // Bs reused by the next piece
    }
  }
  if (ok && region) {
    // this chunk's diagonal block: every earlier block's strip is applied
    // (chunk 0 reads it from K; the others left it in LDS, see above)
    const int j0 = k0 + 64 * c;
    const int bj = ce - j0 < 64 ? ce - j0 : 64;
    if (c == 0)
      diag64_body<true, false, T, false>(K, ld, j0, bj, D, Lb0, info, smem, smem + 64 * DS, smem + 2 * 64 * DS,
                                         nullptr);
    else
      diag64_body<true, false, T, true>(K, ld, j0, bj, D, Lb0 + (int64_t)c * 64 * 64, info, smem, smem + 64 * DS,
                                        smem + 2 * 64 * DS, nullptr);
    if (!(inject && c == 0)) publish(&ctrl[OP_DIAG + c]);  // inject: tests of the timeout path only
  }
  // ---- completion: the last workgroup out zeroes the ctrl words
  __syncthreads();
  if (tid == 0) {
    const unsigned prev = __hip_atomic_fetch_add(&ctrl[OP_DONE], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      for (int i = 0; i < OP_WORDS; ++i)
        if (i != OP_ERR) __hip_atomic_store(&ctrl[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <typename T>
static hipError_t outer_panel_t(T* K, int64_t ld, int N, int k0, int bo, T* D, T* Lb0, T* Wp, int ldw, int* info,
                                unsigned* ctrl, hipStream_t st) {
  if (bo <= 0 || bo > IPMZ_NBO_MAX || k0 + bo > N) return hipErrorInvalidValue;
  const int nch = (N - k0 + 63) / 64;
  hipLaunchKernelGGL(outer_panel_kernel<T>, dim3(nch), dim3(256), 0, st, K, ld, N, k0, k0 + bo, D, Lb0, Wp, ldw, info,
                     ctrl, debug_inject_mask() & IPMZ_INJECT_PANEL);
  return hipGetLastError();
}
hipError_t outer_panel(double* K, int64_t ld, int N, int k0, int bo, double* D, double* Lb0, double* Wp, int ldw,
                       int* info, unsigned* ctrl, hipStream_t st) {
  return outer_panel_t<double>(K, ld, N, k0, bo, D, Lb0, Wp, ldw, info, ctrl, st);
}
hipError_t outer_panel(float* K, int64_t ld, int N, int k0, int bo, float* D, float* Lb0, float* Wp, int ldw,
                       int* info, unsigned* ctrl, hipStream_t st) {
  return outer_panel_t<float>(K, ld, N, k0, bo, D, Lb0, Wp, ldw, info, ctrl, st);
}

}  // namespace ipmz
