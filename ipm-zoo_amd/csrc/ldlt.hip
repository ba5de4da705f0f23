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
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "diag64.h"
#include "kernels.h"

namespace ipmz {

// ---------------------------------------------------------------------------
// Diagonal block (NB x NB, NB in {64, 128}) in REGISTERS.
//
// Thread grid T x T (T = NB/4; NB^2/16 threads), thread (tr, tc) holds the
// 16 elements (tr + T a, tc + T b), a, b in 0..3.  Threads are numbered
// column-major (tid = tc*T + tr), so the owners of one matrix column are T
// consecutive lanes of ONE wave.  Lower-triangle elements hold A -> L; upper
// elements (r < c) hold X^T where X = L^{-1} is built by applying every
// elimination step to the identity (Gauss-Jordan), so the solve and the
// panel TRSM get L11^{-1} for free.
//
// Step k (one workgroup barrier per step):
//   owner wave: d_k from the diagonal owner (readlane), the zero-pivot rule of
//     LinearSolvers.cpp:26-28, publish w_r = A[r][k] (r > k; = l_r d_k),
//     l_r = w_r / d_k, and x_r = X[k][r] (r < k) to LDS (double-buffered by k)
//   everyone: A[r][c] -= l_r w_c (k < c <= r),  X^T[r][c] -= l_c x_r (r <= k < c)
// The update is the reference's  sum -= L[r][k] * L[c][k] * D[k]
// (LinearSolvers.cpp:33) with L[c][k] * D[k] = w_c formed exactly once.
template <typename T, int NB>
__global__ __launch_bounds__(NB* NB / 16) void ldlt_diag_kernel(T* __restrict__ K, int64_t ld, int k0, int b,
                                                                T* __restrict__ D, T* __restrict__ Linv,
                                                                int* __restrict__ info, int64_t sK, int64_t sD,
                                                                int64_t sL) {
  constexpr int TG = NB / 4, NT = TG * TG;
  K += blockIdx.x * sK;  // batch: one workgroup per QP
  D += blockIdx.x * sD;
  Linv += blockIdx.x * sL;
  __shared__ T M[NB][NB + 1];  // coalesced staging in/out
  __shared__ T wsh[2][NB], lsh[2][NB], xsh[2][NB];
  __shared__ T dsh[NB];
  const int tid = threadIdx.x;
  const int tr = tid % TG, tc = tid / TG;
  const int lane = tid & 63, wave = tid >> 6;
  for (int idx = tid; idx < NB * NB; idx += NT) {
    const int r = idx / NB, c = idx % NB;
    M[r][c] = (r < b && c <= r) ? K[(int64_t)(k0 + r) * ld + k0 + c] : (r == c ? T(1) : T(0));
  }
  __syncthreads();
  T v[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) v[a][c4] = M[tr + TG * a][tc + TG * c4];

#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    for (int kk = 0; kk < TG; ++kk) {
      const int k = kb * TG + kk;
      if (k >= b) break;
      const int buf = k & 1;
      const int owner_wave = (kk * TG) >> 6;
      if (wave == owner_wave) {
        const int diag_lane = (kk * TG + kk) & 63;
        const T draw = readlane_t(v[kb][kb], diag_lane);
        const T dk = draw == T(0) ? T(1e-8) : draw;
        const T rdk = T(1) / dk;
        if (tc == kk) {
#pragma unroll
          for (int a = 0; a < 4; ++a) {
            const int r = tr + TG * a;
            const T w = v[a][kb];
            if (r > k) {
              const T l = w * rdk;
              v[a][kb] = l;
              wsh[buf][r] = w;
              lsh[buf][r] = l;
            } else if (r < k) {
              xsh[buf][r] = w;
            } else {
              xsh[buf][r] = T(1);
              dsh[k] = dk;
            }
          }
        }
      }
      __syncthreads();
      T lr[4], xr[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int r = tr + TG * a;
        lr[a] = r > k ? lsh[buf][r] : T(0);
        xr[a] = r <= k ? xsh[buf][r] : T(0);
      }
#pragma unroll
      for (int c4 = kb; c4 < 4; ++c4) {  // columns of blocks < kb are finished
        const int c = tc + TG * c4;
        if (c > k) {
          const T wc = wsh[buf][c], lc = lsh[buf][c];
#pragma unroll
          for (int a = 0; a < 4; ++a) {
            const int r = tr + TG * a;
            if (r >= c) v[a][c4] = fma(-lr[a], wc, v[a][c4]);
            else if (r <= k) v[a][c4] = fma(-lc, xr[a], v[a][c4]);
          }
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c4 = 0; c4 < 4; ++c4) M[tr + TG * a][tc + TG * c4] = v[a][c4];
  __syncthreads();
  // write back L (strict lower), D, and L^{-1} (NB x NB row-major, identity-padded)
  for (int idx = tid; idx < NB * NB; idx += NT) {
    const int r = idx / NB, c = idx % NB;
    if (r < b && c < r) K[(int64_t)(k0 + r) * ld + k0 + c] = M[r][c];
    T x;
    if (r == c) x = T(1);
    else if (c < r && r < b) x = M[c][r];
    else x = T(0);
    Linv[idx] = x;
  }
  for (int k = tid; k < b; k += NT) {
    const T dk = dsh[k];
    D[k0 + k] = dk;
    if (!(fabs((double)dk) <= 1.7976931348623157e308)) atomicMin(info, k0 + k + 1);  // first non-finite pivot
  }
}

// ---------------------------------------------------------------------------
// Diagonal block, NB = 64, ONE wave (the latency-critical kernel of the
// factor: 176 of them sit back to back on the panel path at N = 11264).
//
// Lane r holds row r of the block in 64 registers.  Step k:
//   w_r = A[r][k] goes to LDS (one ds_write per lane, double-buffered by k),
//   d_k = readlane(A[k][k], k), the zero-pivot rule of LinearSolvers.cpp:26-28,
//   l_r = w_r / d_k, then A[r][j] -= l_r w_j for j > k with w_j a broadcast
//   LDS read.  No workgroup barrier anywhere in the 64 steps: a wave's LDS
//   operations complete in order, so a wave-scope fence (no waitcnt) is all
//   the write -> broadcast-read hand-off needs.
// Upper-triangle registers (j > r) carry finite junk that is never read.
// L^{-1} is built afterwards column-per-lane (lane c: L y = e_c, right-looking
// so the 2016 FMAs are independent), reading L^T from LDS by broadcast.
// Same arithmetic as ldlt_diag_kernel: A[r][c] -= l_r * w_c, l = w * (1/d).
template <bool RL, bool INV = true>
__global__ __launch_bounds__(64) void ldlt_diag64_wave_kernel(double* __restrict__ K, int64_t ld, int k0, int b,
                                                              double* __restrict__ D, double* __restrict__ Linv,
                                                              int* __restrict__ info, int64_t sK, int64_t sD,
                                                              int64_t sL) {
  constexpr int S = 66;  // even row stride: M[j][2p..2p+1] is one aligned 16-byte broadcast read
  K += blockIdx.x * sK;
  D += blockIdx.x * sD;
  Linv += blockIdx.x * sL;
  __shared__ __attribute__((aligned(16))) double M[64 * S];
  __shared__ __attribute__((aligned(16))) double wb[2][64];
  const int r = threadIdx.x;
  // coalesced load (lanes over columns): all 64 loads in flight, addresses
  // clamped into the block's valid lower triangle, identity padding past b
  {
    double t[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      const int ii = i < b ? i : 0, cc = r <= ii ? r : 0;
      t[i] = K[(int64_t)(k0 + ii) * ld + k0 + cc];
    }
#pragma unroll
    for (int i = 0; i < 64; ++i) M[i * S + r] = (i < b && r <= i) ? t[i] : (i == r ? 1.0 : 0.0);
  }
  __syncthreads();
  double a[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) a[j] = M[r * S + j];
  double dreg = 1.0;
  static_for<64>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const double wb_self = a[k];
    if constexpr (!RL) wb[k & 1][r] = a[k];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const double draw = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(a[k]), k),
                                         __builtin_amdgcn_readlane(__double2loint(a[k]), k));
    const double dk = draw == 0.0 ? 1e-8 : draw;
    const double rdk = 1.0 / dk;
    dreg = r == k ? dk : dreg;
    const double l = a[k] * rdk;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if constexpr (RL) {  // broadcast w_j straight from lane j's register
      static_for<63 - k>([&](auto jc) {
        constexpr int j = k + 1 + decltype(jc)::value;
        const double wj = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(wb_self), j),
                                           __builtin_amdgcn_readlane(__double2loint(wb_self), j));
        a[j] = fma(-l, wj, a[j]);
      });
      a[k] = l;
      return;
    }
    const double2* w2 = reinterpret_cast<const double2*>(wb[k & 1]);
    // 16 columns per batch: 8 broadcast b128 reads, then 16 independent FMAs
    static_for<4 - (k + 1) / 16>([&](auto cc) {
      constexpr int c0 = ((k + 1) / 16 + decltype(cc)::value) * 16;
      double2 wv[8];
#pragma unroll
      for (int p = 0; p < 8; ++p) wv[p] = w2[c0 / 2 + p];
      static_for<16>([&](auto jc) {
        constexpr int j = c0 + decltype(jc)::value;
        if constexpr (j > k) a[j] = fma(-l, (j & 1) ? wv[(j - c0) / 2].y : wv[(j - c0) / 2].x, a[j]);
      });
    });
    a[k] = l;
  });
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 64; ++j) M[j * S + r] = a[j];  // M[j][i] = L[i][j] for i > j
  __syncthreads();
#pragma unroll 8
  for (int i = 1; i < 64; ++i)
    if (i < b && r < i) K[(int64_t)(k0 + i) * ld + k0 + r] = M[r * S + i];
  if (r < b) {
    D[k0 + r] = dreg;
    if (!(fabs(dreg) <= 1.7976931348623157e308)) atomicMin(info, k0 + r + 1);  // first non-finite pivot
  }
  if constexpr (!INV) return;
  // lane c: column c of L^{-1}, right-looking (y[i] -= L[i][j] y[j], i > j)
  double y[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) y[i] = i == r ? 1.0 : 0.0;
  static_for<63>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const double2* l2 = reinterpret_cast<const double2*>(&M[j * S]);
    static_for<4 - (j + 1) / 16>([&](auto cc) {
      constexpr int c0 = ((j + 1) / 16 + decltype(cc)::value) * 16;
      double2 lv[8];
#pragma unroll
      for (int p = 0; p < 8; ++p) lv[p] = l2[c0 / 2 + p];
      static_for<16>([&](auto ic) {
        constexpr int i = c0 + decltype(ic)::value;
        if constexpr (i > j) y[i] = fma(-((i & 1) ? lv[(i - c0) / 2].y : lv[(i - c0) / 2].x), y[j], y[i]);
      });
    });
  });
#pragma unroll
  for (int i = 0; i < 64; ++i) Linv[i * 64 + r] = y[i];
}

__device__ unsigned long long g_diag_clk[32];
template <bool PROF = false>
__global__ __launch_bounds__(256) void ldlt_diag64_blk_kernel(double* __restrict__ K, int64_t ld, int k0, int b,
                                                              double* __restrict__ D, double* __restrict__ Linv,
                                                              int* __restrict__ info, int64_t sK, int64_t sD,
                                                              int64_t sL) {
  __shared__ double M[64 * DS], X[64 * DS], dsh[64];
  diag64_body<false>(K + blockIdx.x * sK, ld, k0, b, D + blockIdx.x * sD, Linv + blockIdx.x * sL, info, M, X, dsh,
                     PROF ? g_diag_clk : nullptr);
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

template <typename T>
struct GemmArgsT {
  int M, N, Kd;
  const T* A;
  int64_t lda;
  const T* B;
  int64_t ldb;
  T* C;
  int64_t ldc;
  // EPI_PANEL: W[i][j] = acc, C[i][j] = acc / dvec[j]
  T* W;
  int64_t ldw;
  const T* dvec;
  // lower-triangle restriction: tile skipped when row0+gi_end <= col0+gj_start
  int64_t row0, col0;
  int lower;  // 0: full rectangle, 1: skip strictly-upper tiles, 2: triangular grid (row0==col0, BM==BN)
  int ntm, ntn;
  // batch (blockIdx.y = QP): element strides between the QPs' operands
  int64_t sA, sB, sC, sW, sD;
};
using GemmArgs = GemmArgsT<double>;

// Tile pipeline: one LDS buffer is computed while the next k-chunk sits in
// registers (loads issued before the MFMAs, written to the other buffer
// after them): one barrier per 16-deep k-chunk.
template <typename T, int BM, int BN, int NTH>
struct TileLoader {
  typedef typename Mfma<T>::vec2_t V2;
  static constexpr int BK = 16, PAD = 18;
  static constexpr int QA = BM * BK / 2 / NTH, QB = BN * BK / 2 / NTH;  // double2 per thread
  V2 ra[QA], rb[QB];
  __device__ __forceinline__ void load(const GemmArgsT<T>& g, int i0, int j0, int kk) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int ch = tid + NTH * q, r = ch >> 3, c = (ch & 7) * 2;
      ra[q] = fetch(g.A, g.lda, i0 + r, g.M, kk + c, g.Kd);
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int ch = tid + NTH * q, r = ch >> 3, c = (ch & 7) * 2;
      rb[q] = fetch(g.B, g.ldb, j0 + r, g.N, kk + c, g.Kd);
    }
  }
  __device__ __forceinline__ void store(T* As, T* Bs) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int ch = tid + NTH * q, r = ch >> 3, c = (ch & 7) * 2;
      *reinterpret_cast<V2*>(&As[r * PAD + c]) = ra[q];
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int ch = tid + NTH * q, r = ch >> 3, c = (ch & 7) * 2;
      *reinterpret_cast<V2*>(&Bs[r * PAD + c]) = rb[q];
    }
  }
  static __device__ __forceinline__ V2 fetch(const T* P, int64_t ld, int row, int rows, int k, int Kd) {
    V2 t;
    t.x = T(0);
    t.y = T(0);
    if (row < rows) {
      const T* p = P + (int64_t)row * ld + k;
      if (k + 1 < Kd) t = *reinterpret_cast<const V2*>(p);
      else if (k < Kd) t.x = p[0];
    }
    return t;
  }
};

// OPT bits:
//   OPT_NOR2  LDS offsets laundered per k-step so the compiler cannot fuse
//             two reads into ds_read2_b64 (its 16-lane, mod-32 banking turns
//             the PAD = 18 rows into 2-way conflicts; ds_read_b64 is
//             conflict-free)
//   OPT_GRP   grouped triangular enumeration: bands of GRP tile rows walked
//             column by column, so an XCD's ~64 resident tiles share ~8 W and
//             ~8 L row panels in its L2 instead of one W and ~64 L panels
enum { OPT_NOR2 = 2, OPT_GRP = 4 };
constexpr int GRP = 8;

// grouped enumeration of the lower tiles (tm >= tn) of an ntm x ntm grid
__device__ __forceinline__ void grouped_tile(int bid, int ntm, int& tm, int& tn) {
  int r = (int)((sqrt(8.0 * (double)bid + 1.0) - 1.0) * 0.5);
  while ((r + 1) * (r + 2) / 2 <= bid) ++r;
  while (r * (r + 1) / 2 > bid) --r;
  const int b0 = (r / GRP) * GRP;              // first row of the band
  const int gb = ntm - b0 < GRP ? ntm - b0 : GRP;  // rows in the band
  int li = bid - b0 * (b0 + 1) / 2;
  if (li < b0 * gb) {  // rectangular part: columns < b0, gb rows each
    tn = li / gb;
    tm = b0 + li % gb;
    return;
  }
  li -= b0 * gb;
  for (int t = 0;; ++t) {  // triangular part: column b0 + t has rows b0 + t .. b0 + gb - 1
    const int cnt = gb - t;
    if (li < cnt) {
      tn = b0 + t;
      tm = b0 + t + li;
      return;
    }
    li -= cnt;
  }
}

// 8-wave tiles are sized for two workgroups per CU = 4 waves per SIMD, which
// needs <= 128 VGPRs: pinned with amdgpu_waves_per_eu (the compiler otherwise
// drifts to 129+ and silently halves the occupancy)
template <typename T, int BM, int BN, int EPI, int WGM = 2, int WGN = 2, int OPT = OPT_NOR2>
__global__ __launch_bounds__(64 * WGM * WGN)
__attribute__((amdgpu_waves_per_eu(WGM * WGN == 8 ? 4 : 1))) void gemm_nt_kernel(GemmArgsT<T> g) {
  typedef Mfma<T> MF;
  constexpr int BK = 16, PAD = 18, NTH = 64 * WGM * WGN;
  if (blockIdx.y) {
    const int64_t z = blockIdx.y;
    g.A += z * g.sA;
    g.B += z * g.sB;
    g.C += z * g.sC;
    if (EPI == EPI_PANEL) {
      g.W += z * g.sW;
      g.dvec += z * g.sD;
    }
  }
  constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  __shared__ __attribute__((aligned(16))) T As[2][BM * PAD];
  __shared__ __attribute__((aligned(16))) T Bs[2][BN * PAD];

  // XCD-aware remap (cdna_hip_programming.md T1, bijective form): blocks
  // b and b+8 share an XCD, so consecutive logical tiles -- which share W
  // (A) rows in both enumerations -- are handed to one XCD's L2.
  int bid = blockIdx.x;
  {
    const int nwg = gridDim.x, q = nwg / 8, r = nwg % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  int tm, tn;
  if (g.lower == 2) {
    if constexpr ((OPT & OPT_GRP) != 0) {
      grouped_tile(bid, g.ntm, tm, tn);
    } else {
      // triangular enumeration of lower tiles: bid -> (tm >= tn)
      int r = (int)((sqrt(8.0 * (double)bid + 1.0) - 1.0) * 0.5);
      while ((r + 1) * (r + 2) / 2 <= bid) ++r;
      while (r * (r + 1) / 2 > bid) --r;
      tm = r;
      tn = bid - r * (r + 1) / 2;
    }
  } else {
    tn = bid % g.ntn;
    tm = bid / g.ntn;
  }
  const int i0 = tm * BM, j0 = tn * BN;
  if (g.lower == 1 && g.row0 + i0 + BM - 1 < g.col0 + j0) return;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WGN, wc = wave % WGN;
  typename MF::acc_t acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = (typename MF::acc_t){T(0), T(0), T(0), T(0)};

  TileLoader<T, BM, BN, NTH> ld;
  const int nch = (g.Kd + BK - 1) / BK;
  ld.load(g, i0, j0, 0);
  ld.store(As[0], Bs[0]);
  __syncthreads();
  const int aoff = (wr * WM + (lane & 15)) * PAD + (lane >> 4);
  const int boff = (wc * WN + (lane & 15)) * PAD + (lane >> 4);
  for (int t = 0; t < nch; ++t) {
    const int cur = t & 1;
    if (t + 1 < nch) ld.load(g, i0, j0, (t + 1) * BK);
    const T* as = As[cur];
    const T* bs = Bs[cur];
#pragma unroll
    for (int s = 0; s < BK / 4; ++s) {
      int ao = aoff + 4 * s, bo = boff + 4 * s;
      if constexpr ((OPT & OPT_NOR2) != 0) {
        asm volatile("" : "+v"(ao));
        asm volatile("" : "+v"(bo));
      }
      T af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = as[ao + a * 16 * PAD];
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b] = bs[bo + b * 16 * PAD];
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = MF::mma(af[a], bf[b], acc[a][b]);
    }
    if (t + 1 < nch) ld.store(As[cur ^ 1], Bs[cur ^ 1]);
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
        const int i = i0 + wr * WM + a * 16 + MF::row(lane, r);
        if (i < g.M && j < g.N) {
          const T v = acc[a][b][r];
          T* cp = g.C + (int64_t)i * g.ldc + j;
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

template <int BM, int BN, int EPI, int WGM = 2, int WGN = 2, int OPT = OPT_NOR2, typename T = double>
static hipError_t launch_gemm(GemmArgsT<T> g, hipStream_t st, int batch = 1) {
  g.ntm = (g.M + BM - 1) / BM;
  g.ntn = (g.N + BN - 1) / BN;
  if (g.ntm == 0 || g.ntn == 0 || g.Kd == 0) return hipSuccess;
  int64_t nblk = (int64_t)g.ntm * g.ntn;
  if (g.lower == 2) {
    // triangular enumeration needs square tiles; BM = k * BN tiles use a
    // rectangular grid with upper-tile skipping instead
    if (BM == BN) nblk = (int64_t)g.ntm * (g.ntm + 1) / 2;
    else g.lower = 1;
  }
  hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, EPI, WGM, WGN, OPT>), dim3((unsigned)nblk, (unsigned)batch),
                     dim3(64 * WGM * WGN), 0, st, g);
  return hipGetLastError();
}

// experiment hook (kbench): trailing update with a chosen tile variant
hipError_t gemm_nt_sub_variant(int variant, int M, int N, int Kd, const double* A, int64_t lda, const double* B,
                               int64_t ldb, double* C, int64_t ldc, hipStream_t st) {
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
  g.lower = 2;
  switch (variant) {
    case 0: return launch_gemm<128, 128, EPI_SUB>(g, st);
    case 1: return launch_gemm<256, 128, EPI_SUB, 4, 2>(g, st);
    case 2: return launch_gemm<128, 128, EPI_SUB, 2, 4, 0>(g, st);
    case 3: return launch_gemm<128, 64, EPI_SUB, 2, 1>(g, st);
    case 4: return launch_gemm<256, 128, EPI_SUB, 4, 4>(g, st);
    case 5: return launch_gemm<128, 128, EPI_SUB, 4, 4>(g, st);
    case 6: return launch_gemm<128, 256, EPI_SUB, 2, 8>(g, st);
    case 9: return launch_gemm<128, 128, EPI_SUB, 2, 4, OPT_NOR2>(g, st);
    case 10: return launch_gemm<128, 128, EPI_SUB, 2, 4, OPT_GRP>(g, st);  // (these two spill one VGPR)
    case 14: return launch_gemm<128, 128, EPI_SUB, 2, 4, OPT_NOR2 | OPT_GRP>(g, st);
    case 15: return launch_gemm<128, 128, EPI_SUB, 4, 4, OPT_NOR2 | OPT_GRP>(g, st);
    case 16: return launch_gemm<128, 128, EPI_SUB, 4, 4, OPT_GRP>(g, st);
    case 23: return launch_gemm<64, 64, EPI_SUB, 2, 2, OPT_NOR2 | OPT_GRP>(g, st);
    default: break;
  }
  // strip (rectangle, upper tiles of the diagonal band skipped) variants
  g.lower = 1;
  switch (variant) {
    case 20: return launch_gemm<128, 128, EPI_SUB_STRIP, 2, 4, OPT_NOR2>(g, st);
    case 21: return launch_gemm<64, 64, EPI_SUB_STRIP, 2, 2, OPT_NOR2>(g, st);
    case 22: return launch_gemm<64, 128, EPI_SUB_STRIP, 2, 4, OPT_NOR2>(g, st);
    case 24: return launch_gemm<128, 128, EPI_SUB_STRIP, 4, 4, OPT_NOR2>(g, st);
    case 25: return launch_gemm<64, 128, EPI_SUB_STRIP, 4, 4, OPT_NOR2>(g, st);
    case 26: return launch_gemm<64, 64, EPI_SUB_STRIP, 4, 4, OPT_NOR2>(g, st);
    default: return hipErrorInvalidValue;
  }
}

// experiment hooks (kbench): one diag block, one panel TRSM
// diag kernel choice for nbi = 64: 5 = MFMA-blocked diag64_body (default), 0 = 4-wave barrier-per-step,
// 1 = one wave with LDS broadcasts, 2 = one wave with readlane broadcasts
static int diag64_variant() {
  static const int v = [] {
    const char* e = std::getenv("IPMZ_DIAG");
    if (!e) return 5;  // MFMA-blocked (C4 batch 128: factor 0.35 -> 0.26 ms)
    if (!std::strcmp(e, "reg")) return 0;
    if (!std::strcmp(e, "wave")) return 1;
    if (!std::strcmp(e, "wave_rl")) return 2;
    if (!std::strcmp(e, "blk")) return 5;
    return 0;
  }();
  return v;
}
static void launch_diag64(int variant, int B, hipStream_t st, double* K, int64_t ld, int j0, int bi, double* D,
                          double* Lb, int* info, int64_t sK, int64_t sD, int64_t sL) {
  if (variant == 5)
    hipLaunchKernelGGL(ldlt_diag64_blk_kernel<false>, dim3(B), dim3(256), 0, st, K, ld, j0, bi, D, Lb, info, sK, sD, sL);
  else if (variant == 1)
    hipLaunchKernelGGL(ldlt_diag64_wave_kernel<false>, dim3(B), dim3(64), 0, st, K, ld, j0, bi, D, Lb, info, sK, sD, sL);
  else if (variant == 2)
    hipLaunchKernelGGL(ldlt_diag64_wave_kernel<true>, dim3(B), dim3(64), 0, st, K, ld, j0, bi, D, Lb, info, sK, sD, sL);
  else if (variant == 3)  // timing probes: no L^{-1}
    hipLaunchKernelGGL((ldlt_diag64_wave_kernel<false, false>), dim3(B), dim3(64), 0, st, K, ld, j0, bi, D, Lb, info, sK,
                       sD, sL);
  else if (variant == 4)
    hipLaunchKernelGGL((ldlt_diag64_wave_kernel<true, false>), dim3(B), dim3(64), 0, st, K, ld, j0, bi, D, Lb, info, sK,
                       sD, sL);
  else
    hipLaunchKernelGGL((ldlt_diag_kernel<double, 64>), dim3(B), dim3(256), 0, st, K, ld, j0, bi, D, Lb, info, sK, sD, sL);
}

// fp32 factor (mixed-precision path): the register-resident 4-wave kernel
static void launch_diag64(int, int B, hipStream_t st, float* K, int64_t ld, int j0, int bi, float* D, float* Lb,
                          int* info, int64_t sK, int64_t sD, int64_t sL) {
  hipLaunchKernelGGL((ldlt_diag_kernel<float, 64>), dim3(B), dim3(256), 0, st, K, ld, j0, bi, D, Lb, info, sK, sD, sL);
}

// stage clock (s_memtime) of one ldlt_diag64_blk_kernel run, for kbench
hipError_t diag_clock_probe(double* K, int64_t ld, double* D, double* Linv, int* info, unsigned long long* out,
                            hipStream_t st) {
  hipLaunchKernelGGL(ldlt_diag64_blk_kernel<true>, dim3(1), dim3(256), 0, st, K, ld, 0, 64, D, Linv, info, 0, 0, 0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return hipMemcpyFromSymbolAsync(out, HIP_SYMBOL(g_diag_clk), sizeof(unsigned long long) * 32, 0,
                                  hipMemcpyDeviceToHost, st);
}

hipError_t diag_probe(double* K, int64_t ld, int k0, int nbi, double* D, double* Linv, int* info, hipStream_t st) {
  if (nbi == 128)
    hipLaunchKernelGGL((ldlt_diag_kernel<double, 128>), dim3(1), dim3(1024), 0, st, K, ld, k0, nbi, D, Linv, info, 0, 0, 0);
  else  // nbi = -variant - 64 .. : kernel variants at 64
    launch_diag64(nbi <= -64 ? -nbi - 64 : 0, 1, st, K, ld, k0, 64, D, Linv, info, 0, 0, 0);
  return hipGetLastError();
}
hipError_t trsm_probe(double* K, int64_t ld, int N, int j0, double* D, const double* Linv, double* W, int nbo,
                      hipStream_t st) {
  const int r1 = j0 + 64;
  GemmArgs g{};
  g.M = N - r1;
  g.N = 64;
  g.Kd = 64;
  g.A = K + (int64_t)r1 * ld + j0;
  g.lda = ld;
  g.B = Linv;
  g.ldb = 64;
  g.C = K + (int64_t)r1 * ld + j0;
  g.ldc = ld;
  g.W = W + (int64_t)r1 * nbo;
  g.ldw = nbo;
  g.dvec = D + j0;
  return launch_gemm<128, 64, EPI_PANEL, 4, 2>(g, st);
}

// f64 MFMA throughput probe: each wave runs `iters` x 16 independent
// v_mfma_f64_16x16x4 on register data.
template <int NACC>
__global__ __launch_bounds__(512) void mfma_probe_kernel(double* out, int iters) {
  double4_t acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = (double4_t){0.0, 0.0, 0.0, 0.0};
  double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = mfma_f64_16x16x4(a, b, acc[i]);
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[0] = s;
}
// waves_per_simd in {1, 2}: 256- or 512-thread blocks, one block per CU
hipError_t mfma_probe(double* out, int blocks, int iters, int threads, int nacc, hipStream_t st) {
  if (nacc == 16) hipLaunchKernelGGL(mfma_probe_kernel<16>, dim3(blocks), dim3(threads), 0, st, out, iters);
  else if (nacc == 8) hipLaunchKernelGGL(mfma_probe_kernel<8>, dim3(blocks), dim3(threads), 0, st, out, iters);
  else if (nacc == 2) hipLaunchKernelGGL(mfma_probe_kernel<2>, dim3(blocks), dim3(threads), 0, st, out, iters);
  else if (nacc == 1) hipLaunchKernelGGL(mfma_probe_kernel<1>, dim3(blocks), dim3(threads), 0, st, out, iters);
  else hipLaunchKernelGGL(mfma_probe_kernel<4>, dim3(blocks), dim3(threads), 0, st, out, iters);
  return hipGetLastError();
}

// C[i][j] -= sum_k A[i][k] B[j][k] over the lower part of a trailing region.
template <typename T>
static hipError_t gemm_nt_sub_t(int M, int N, int Kd, const T* A, int64_t lda, const T* B, int64_t ldb, T* C,
                                int64_t ldc, int64_t row0, int64_t col0, bool square_lower, hipStream_t st,
                                const BatchStrides* bs) {
  GemmArgsT<T> g{};
  int batch = 1;
  if (bs && bs->B > 1) {
    batch = bs->B;
    g.sA = bs->sW;  // A is a W panel, B and C live in K
    g.sB = bs->sK;
    g.sC = bs->sK;
  }
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
  // 128x128 tile, 8 waves as 2 x 4 (64 x 32 per wave, 128 VGPRs), 72 KB LDS:
  // two workgroups per CU = 4 waves per SIMD (kbench: 47 TFLOP/s = 60 % of
  // the fp64 MFMA peak at R = 11008, vs 25 with 4 waves of 64 x 64)
  // ds_read_b64 without read2 fusion + grouped tile order: 53 vs 48 TFLOP/s
  // (kbench, R = 11008, rank 256).  Small updates -- the look-ahead strip and
  // the trailing updates of the last panels, all latency-bound -- take
  // 64-wide tiles: 4x the workgroups, a quarter of the work per k-chunk
  // (kbench rank 256: strip M = 4096 46 -> 24 us, trailing R = 1536 51 -> 34 us)
  // fp64 trailing update: 16 waves as 4 x 4 (32 x 32 per wave, 64 VGPRs,
  // two workgroups = 32 waves per CU): 56.6 vs 55.2 TFLOP/s alone (kbench
  // gvar, R = 10880, rank 384), 40.8 vs 38.9 in situ, C3 60.6 -> 61.8
  // steps/s; the fp32 factor (C5) keeps 2 x 4 (71 vs 67 TFLOP/s in situ)
  if (square_lower) {
    if (M <= IPMZ_TRAIL_SMALL_M) return launch_gemm<64, 64, EPI_SUB, 2, 2, OPT_NOR2 | OPT_GRP>(g, st, batch);
    if constexpr (std::is_same<T, double>::value)
      return launch_gemm<128, 128, EPI_SUB, 4, 4, OPT_NOR2 | OPT_GRP>(g, st, batch);
    return launch_gemm<128, 128, EPI_SUB, 2, 4, OPT_NOR2 | OPT_GRP>(g, st, batch);
  }
  if (M <= 4096) return launch_gemm<64, 64, EPI_SUB_STRIP, 2, 2, OPT_NOR2>(g, st, batch);
  if (M <= 8192) return launch_gemm<64, 128, EPI_SUB_STRIP, 2, 4, OPT_NOR2>(g, st, batch);
  return launch_gemm<128, 128, EPI_SUB_STRIP, 2, 4, OPT_NOR2>(g, st, batch);
}
hipError_t gemm_nt_sub(int M, int N, int Kd, const double* A, int64_t lda, const double* B, int64_t ldb,
                       double* C, int64_t ldc, int64_t row0, int64_t col0, bool square_lower, hipStream_t st,
                       const BatchStrides* bs) {
  return gemm_nt_sub_t<double>(M, N, Kd, A, lda, B, ldb, C, ldc, row0, col0, square_lower, st, bs);
}

hipError_t gemm_nt_sub_rect(int M, int N, int Kd, const double* A, int64_t lda, const double* B, int64_t ldb,
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
  return launch_gemm<128, 128, EPI_SUB_STRIP, 2, 4>(g, st);
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
  return launch_gemm<128, 128, EPI_STORE, 2, 4>(g, st);
}

// ---------------------------------------------------------------------------
// Factor the outer panel [k0, k0 + bo): inner diag / TRSM / strip steps, all
// on stream st.  Writes L (in K), D, the L11^{-1} blocks and W = L D for
// the panel's rows below each inner block (W: N x nbo, this panel's buffer).
// panel path: 2 = the whole outer panel in one launch (default), 1 = one
// fused launch per inner block (IPMZ_PANEL=step), 0 = diag / TRSM / strip
// kernel chain (IPMZ_PANEL=chain)
static int panel_mode() {
  static const int mode = [] {
    const char* e = std::getenv("IPMZ_PANEL");
    if (e && !std::strcmp(e, "chain")) return 0;
    if (e && !std::strcmp(e, "step")) return 1;
    return 2;
  }();
  return mode;
}

// fused panel kernels (fp64): one launch per outer panel / per inner block
static hipError_t fused_panel(double* K, int64_t ld, int N, double* D, double* Linv, double* W, int k0, int bo, int nbo,
                              int nbi, int* info, unsigned* pctrl, hipStream_t st) {
  if (panel_mode() == 2)
    return outer_panel(K, ld, N, k0, bo, D, Linv + (int64_t)(k0 / nbi) * nbi * nbi, W, nbo, info, pctrl, st);
  hipError_t e = hipSuccess;
  for (int j0 = k0; j0 < k0 + bo && e == hipSuccess; j0 += nbi) {
    const int bi = k0 + bo - j0 < nbi ? k0 + bo - j0 : nbi;
    e = panel_step(K, ld, N, j0, bi, k0 + bo, D, Linv + (int64_t)(j0 / nbi) * nbi * nbi, W + (j0 - k0), nbo, info,
                   pctrl, st);
  }
  return e;
}
static hipError_t fused_panel(float* K, int64_t ld, int N, float* D, float* Linv, float* W, int k0, int bo, int nbo,
                              int nbi, int* info, unsigned* pctrl, hipStream_t st) {
  if (panel_mode() != 2) return hipErrorInvalidValue;  // fp32: outer-panel kernel only
  return outer_panel(K, ld, N, k0, bo, D, Linv + (int64_t)(k0 / nbi) * nbi * nbi, W, nbo, info, pctrl, st);
}

template <typename T>
static hipError_t factor_panel(T* K, int64_t ld, int N, T* D, T* Linv, T* W, int k0, int bo, int nbo, int nbi,
                               int* info, hipStream_t st, const BatchStrides* bs = nullptr, unsigned* pctrl = nullptr) {
  hipError_t e = hipSuccess;
  const int B = bs ? bs->B : 1;
  const int64_t sK = bs ? bs->sK : 0, sD = bs ? bs->sD : 0, sL = bs ? bs->sL : 0, sW = bs ? bs->sW : 0;
  if (pctrl && B == 1 && nbi == 64 && (panel_mode() == 2 || (std::is_same<T, double>::value && panel_mode() == 1)))
    return fused_panel(K, ld, N, D, Linv, W, k0, bo, nbo, nbi, info, pctrl, st);
  for (int j0 = k0; j0 < k0 + bo; j0 += nbi) {
    const int bi = k0 + bo - j0 < nbi ? k0 + bo - j0 : nbi;
    T* Lb = Linv + (int64_t)(j0 / nbi) * nbi * nbi;
    if (nbi == 128)
      hipLaunchKernelGGL((ldlt_diag_kernel<T, 128>), dim3(B), dim3(1024), 0, st, K, ld, j0, bi, D, Lb, info, sK, sD, sL);
    else
      launch_diag64(diag64_variant(), B, st, K, ld, j0, bi, D, Lb, info, sK, sD, sL);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const int r1 = j0 + bi;
    if (r1 >= N) continue;
    // panel TRSM: rows [r1, N): T = A21 L11^{-T}, W21 = T, L21 = T / D1
    GemmArgsT<T> g{};
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
    g.sA = sK;
    g.sB = sL;
    g.sC = sK;
    g.sW = sW;
    g.sD = sD;
    e = nbi == 128 ? launch_gemm<128, 128, EPI_PANEL, 2, 4>(g, st, B) : launch_gemm<128, 64, EPI_PANEL, 4, 2>(g, st, B);
    if (e != hipSuccess) return e;
    // strip update of the remaining columns of this outer panel
    const int c1 = k0 + bo;
    if (r1 < c1) {
      e = gemm_nt_sub_t<T>(N - r1, c1 - r1, bi, W + (int64_t)r1 * nbo + (j0 - k0), nbo, K + (int64_t)r1 * ld + j0, ld,
                           K + (int64_t)r1 * ld + r1, ld, r1, r1, false, st, bs);
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

// Rank-bo update of the column block [c0, c1) (rows >= c0) with outer panel
// k (W_k rows, L_k = K[:, k0:k0+bo)); square = the whole trailing triangle.
template <typename T>
static hipError_t panel_update(T* K, int64_t ld, int N, const T* Wk, int nbo, int k0, int bo, int c0, int c1,
                               bool square, hipStream_t st, const BatchStrides* bs = nullptr) {
  if (c0 >= c1 || c0 >= N) return hipSuccess;
  return gemm_nt_sub_t<T>(N - c0, c1 - c0, bo, Wk + (int64_t)c0 * nbo, nbo, K + (int64_t)c0 * ld + k0, ld,
                     K + (int64_t)c0 * ld + c0, ld, c0, c0, square, st, bs);
}

// Batch of B independent factorizations (same N), single stream: each
// launch covers every QP (grid.y / grid.x = QP).  For small N (C4: 320).
hipError_t ldlt_factor_batched(double* K, int64_t ld, int N, double* D, double* Linv, double* W, int nbo, int nbi,
                               int* info, hipStream_t st, const BatchStrides& bs) {
  if (N <= 0 || bs.B <= 0) return hipSuccess;
  if (nbi != 64 && nbi != 128) return hipErrorInvalidValue;
  if (nbo % nbi != 0 || nbo > IPMZ_NBO_MAX) return hipErrorInvalidValue;
  // small systems (C4): the whole factor in one workgroup per QP (small.hip)
  static const bool small_ok = [] {
    const char* e = std::getenv("IPMZ_SMALL");
    return !(e && !std::strcmp(e, "0"));
  }();
  if (small_ok && nbi == 64 && N <= IPMZ_SMALL_NMAX) return ldlt_factor_small_batched(K, ld, N, D, Linv, W, info, st, bs);
  hipError_t e = hipSuccess;
  for (int k0 = 0; k0 < N; k0 += nbo) {
    const int bo = N - k0 < nbo ? N - k0 : nbo, t0 = k0 + bo;
    if ((e = factor_panel(K, ld, N, D, Linv, W, k0, bo, nbo, nbi, info, st, &bs)) != hipSuccess) return e;
    if (t0 < N && (e = panel_update(K, ld, N, W, nbo, k0, bo, t0, N, true, st, &bs)) != hipSuccess) return e;
  }
  return hipSuccess;
}

// Blocked LDL^T with depth-1 look-ahead on two streams (Ws: 3 buffers of
// N x nbo).  With P_k the k-th outer panel:
//   stream A (st): [wait N_{k-1}] update P_{k+1} with P_k ; factor P_{k+1}
//   stream B (st2): [wait P_k] update P_{k+2} with P_k -> event N_k ;
//                   update everything beyond P_{k+2} with P_k (the big
//                   trailing GEMM, overlapping A's panel factorization)
// Correctness: P_{k+1}'s columns get panel j <= k-1 contributions from B
// (ordered on B before N_{k-1}) and panel k's from A; B never touches the
// columns A is factoring; W is triple-buffered so A's P_{k+1} never
// overwrites the W_{k-2} a late B_{k-2} could still read (B_{k-2} precedes
// N_{k-1} on B).  A waits for B's tail at the end.
template <typename T>
static hipError_t ldlt_factor_t(T* K, int64_t ld, int N, T* D, T* Linv, T* W, int nbo, int nbi, int* info,
                                hipStream_t st, TrailTimer* timer, hipStream_t st2, hipEvent_t* ev, int nev,
                                unsigned* pctrl) {
  if (N <= 0) return hipSuccess;
  if (nbi != 64 && nbi != 128) return hipErrorInvalidValue;
  if (nbo % nbi != 0 || nbo > IPMZ_NBO_MAX) return hipErrorInvalidValue;
  const int npan = (N + nbo - 1) / nbo;
  const bool two = st2 != nullptr && ev != nullptr && nev >= 2 * npan + 2;
  const int64_t wsz = (int64_t)N * nbo;
  auto Wb = [&](int k) { return W + (two ? (k % 3) : 0) * wsz; };  // T*
  auto pw = [&](int k) { return N - k * nbo < nbo ? N - k * nbo : nbo; };
  hipError_t e = factor_panel(K, ld, N, D, Linv, Wb(0), 0, pw(0), nbo, nbi, info, st, nullptr, pctrl);
  if (e != hipSuccess) return e;
  if (!two) {  // single stream: factor, then the whole trailing update
    for (int k = 0; k < npan; ++k) {
      const int k0 = k * nbo, bo = pw(k), t0 = k0 + bo;
      if (t0 < N) {
        // timed: the launches of the dominant 128 x 128 trailing kernel
        hipEvent_t* te = timer && N - t0 > IPMZ_TRAIL_SMALL_M ? timer->next() : nullptr;
        if (te) hipEventRecord(te[0], st);
        e = panel_update(K, ld, N, Wb(k), nbo, k0, bo, t0, N, true, st);
        if (te) hipEventRecord(te[1], st);
        if (te) timer->flops += (double)(N - t0) * (double)(N - t0 + 1) * (double)bo;
        if (e != hipSuccess) return e;
        if ((e = factor_panel(K, ld, N, D, Linv, Wb(k + 1), t0, pw(k + 1), nbo, nbi, info, st, nullptr, pctrl)) != hipSuccess)
          return e;
      }
    }
    return hipSuccess;
  }
  hipEvent_t* evP = ev;         // panel k factored (A)
  hipEvent_t* evN = ev + npan;  // P_{k+2} updated with P_k (B)
  hipEvent_t evJoin = ev[2 * npan];
  for (int k = 0; k < npan; ++k) {
    const int k0 = k * nbo, bo = pw(k);
    const int p1 = k0 + bo;                          // start of P_{k+1}
    const int p2 = p1 < N ? p1 + pw(k + 1) : N;      // start of P_{k+2}
    const int p3 = p2 < N ? p2 + pw(k + 2) : N;      // start of P_{k+3}
    if (p1 >= N) break;
    if ((e = hipEventRecord(evP[k], st)) != hipSuccess) return e;
    // ---- stream B: P_{k+2} columns first, then the rest
    if ((e = hipStreamWaitEvent(st2, evP[k], 0)) != hipSuccess) return e;
    if (p2 < N) {
      if ((e = panel_update(K, ld, N, Wb(k), nbo, k0, bo, p2, p3, false, st2)) != hipSuccess) return e;
    }
    if ((e = hipEventRecord(evN[k], st2)) != hipSuccess) return e;
    if (p3 < N) {
      hipEvent_t* te = timer && N - p3 > IPMZ_TRAIL_SMALL_M ? timer->next() : nullptr;
      if (te) hipEventRecord(te[0], st2);
      e = panel_update(K, ld, N, Wb(k), nbo, k0, bo, p3, N, true, st2);
      if (te) hipEventRecord(te[1], st2);
      if (te) timer->flops += (double)(N - p3) * (double)(N - p3 + 1) * (double)bo;
      if (e != hipSuccess) return e;
    }
    // ---- stream A: update P_{k+1} with P_k, factor P_{k+1}
    if (k >= 1) {
      if ((e = hipStreamWaitEvent(st, evN[k - 1], 0)) != hipSuccess) return e;
    }
    if ((e = panel_update(K, ld, N, Wb(k), nbo, k0, bo, p1, p2, false, st)) != hipSuccess) return e;
    if ((e = factor_panel(K, ld, N, D, Linv, Wb(k + 1), p1, pw(k + 1), nbo, nbi, info, st, nullptr, pctrl)) != hipSuccess)
      return e;
  }
  if ((e = hipEventRecord(evJoin, st2)) != hipSuccess) return e;
  return hipStreamWaitEvent(st, evJoin, 0);
}

hipError_t ldlt_factor(double* K, int64_t ld, int N, double* D, double* Linv, double* W, int nbo, int nbi,
                       int* info, hipStream_t st, TrailTimer* timer, hipStream_t st2, hipEvent_t* ev, int nev,
                       unsigned* pctrl) {
  return ldlt_factor_t<double>(K, ld, N, D, Linv, W, nbo, nbi, info, st, timer, st2, ev, nev, pctrl);
}
hipError_t ldlt_factor(float* K, int64_t ld, int N, float* D, float* Linv, float* W, int nbo, int nbi, int* info,
                       hipStream_t st, TrailTimer* timer, hipStream_t st2, hipEvent_t* ev, int nev, unsigned* pctrl) {
  return ldlt_factor_t<float>(K, ld, N, D, Linv, W, nbo, nbi, info, st, timer, st2, ev, nev, pctrl);
}

}  // namespace ipmz
