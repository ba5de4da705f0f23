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
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "common.h"
#include "diag64.h"
#include "gemm.h"
#include "gemm32.h"
#include "gemm64.h"
#include "kernels.h"

namespace ipmz {

static int g_inject = 0;

int debug_inject_mask() { return g_inject; }
void set_debug_inject_mask(int mask) { g_inject = mask; }

// ---------------------------------------------------------------------------
// Capture-safe cross-stream ordering.  The HIP runtime torch bundles
// (7.0.51831; libipmz shares it when loaded after torch) recurses without end
// inside hipStreamEndCapture once two side streams of a capture have waited on
// each other's events -- the look-ahead's chain / rows / trailing streams do
// that every panel (tools/dbg/graph_mini.cpp patterns 2 and 5 crash; 0, 1, 3,
// 6, 7 do not; /opt/rocm's 7.2 captures all of them).  So while a stream is
// capturing, stream_record notes the nodes an event stands for, and
// stream_wait between side streams adds those nodes to the waiter's capture
// dependencies (hipStreamUpdateCaptureDependencies) instead of waiting on the
// event: the same graph edges, no stream-to-stream wait.  A stream joining the
// capture (its first wait) and the capture's origin stream (set_capture_origin)
// wait on the event as usual.  Outside a capture both are the plain calls.
namespace {
struct Noted {
  unsigned long long id;
  std::vector<hipGraphNode_t> nodes;
};
thread_local std::unordered_map<hipEvent_t, Noted> t_noted;
thread_local hipStream_t t_origin = nullptr;
}  // namespace
void set_capture_origin(hipStream_t s) {
  t_origin = s;
  t_noted.clear();
}
hipError_t stream_record(hipEvent_t e, hipStream_t s) {
  hipError_t r = hipEventRecord(e, s);
  if (r != hipSuccess) return r;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if ((r = hipStreamIsCapturing(s, &cs)) != hipSuccess) return r;
  if (cs != hipStreamCaptureStatusActive) {
    t_noted.erase(e);
    return hipSuccess;
  }
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t n = 0;
  if ((r = hipStreamGetCaptureInfo_v2(s, &cs, &id, &g, &deps, &n)) != hipSuccess) return r;
  t_noted[e] = Noted{id, std::vector<hipGraphNode_t>(deps, deps + n)};
  return hipSuccess;
}
hipError_t stream_wait(hipStream_t s, hipEvent_t e) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  hipError_t r = hipStreamIsCapturing(s, &cs);
  if (r != hipSuccess) return r;
  auto it = t_noted.find(e);
  if (cs != hipStreamCaptureStatusActive || s == t_origin || it == t_noted.end()) return hipStreamWaitEvent(s, e, 0);
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t n = 0;
  if ((r = hipStreamGetCaptureInfo_v2(s, &cs, &id, &g, &deps, &n)) != hipSuccess) return r;
  if (id != it->second.id) return hipStreamWaitEvent(s, e, 0);
  if (it->second.nodes.empty()) return hipSuccess;
  return hipStreamUpdateCaptureDependencies(s, it->second.nodes.data(), it->second.nodes.size(),
                                            hipStreamAddCaptureDependencies);
}

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
  const int wave = tid >> 6;
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

// Diagonal block, NB = 64, on fp64 MFMA (diag64.h): the default diagonal
// factor of the kernel-chain panel path (batched factors, nbi = 64).
__global__ __launch_bounds__(256) void ldlt_diag64_blk_kernel(double* __restrict__ K, int64_t ld, int k0, int b,
                                                              double* __restrict__ D, double* __restrict__ Linv,
                                                              int* __restrict__ info, int64_t sK, int64_t sD,
                                                              int64_t sL) {
  __shared__ double M[64 * DS], X[64 * DS], dsh[64];
  diag64_body<false>(K + blockIdx.x * sK, ld, k0, b, D + blockIdx.x * sD, Linv + blockIdx.x * sL, info, M, X, dsh,
                     nullptr);
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

static void launch_diag64(int B, hipStream_t st, double* K, int64_t ld, int j0, int bi, double* D, double* Lb,
                          int* info, int64_t sK, int64_t sD, int64_t sL) {
  hipLaunchKernelGGL(ldlt_diag64_blk_kernel, dim3(B), dim3(256), 0, st, K, ld, j0, bi, D, Lb, info, sK, sD, sL);
}
// fp32 factor (mixed-precision path): the register-resident 4-wave kernel
static void launch_diag64(int B, hipStream_t st, float* K, int64_t ld, int j0, int bi, float* D, float* Lb, int* info,
                          int64_t sK, int64_t sD, int64_t sL) {
  hipLaunchKernelGGL((ldlt_diag_kernel<float, 64>), dim3(B), dim3(256), 0, st, K, ld, j0, bi, D, Lb, info, sK, sD, sL);
}

// ---------------------------------------------------------------------------
// The fp32 updates of the mixed-precision factor (C5) on the 32 x 32 x 2 f32
// MFMA kernel of gemm32.h: the trailing triangle as ONE launch over its lower
// tiles (the round-3 rocBLAS halving tree of strided-batched SGEMMs is gone),
// and the look-ahead strips.  Tile choice by size (tools/sgemm_bench.cpp,
// profiles/r04_*/sgemm*.log).  Operands whose rows are not 16-byte aligned
// (never the factor's own: ld and nbo are multiples of 64) take the gemm.h
// engine; so does debug bit IPMZ_DEBUG_F32_ENGINE (A/B).
static bool sgemm_sub(GemmArgsT<float>& g, bool square_lower, hipStream_t st, hipError_t& e) {
  if (!sgemm_aligned(g) || (debug_inject_mask() & IPMZ_DEBUG_F32_ENGINE)) return false;
  // (profiles/r04_s2: the LDS-DMA tiles against the register-staged ones in
  // the step, C5 44.7 vs 42.7 steps/s)
  if (square_lower) {
    if (g.M <= IPMZ_TRAIL_SMALL_M) e = launch_sgemm<64, 64, 2, 2, 32, 4>(g, st);
    else e = launch_sgemm<128, 128, 2, 2, 16, 2, EPI_SUB, 3, true>(g, st);
    return true;
  }
  if (g.M <= 4096) e = launch_sgemm<64, 64, 2, 2, 32, 4, EPI_SUB_STRIP>(g, st);
  else e = launch_sgemm<128, 128, 2, 4, 16, 4, EPI_SUB_STRIP, 2, true>(g, st);
  return true;
}

// fp64 updates with LDS-DMA staging (gemm64.h) where every tile is full:
// false -- not launched (partial tiles, debug bit IPMZ_DEBUG_F64_ENGINE): the
// caller takes gemm.h's kernel.  In the step: C3 70.7 -> 74.0 steps/s, the
// strips' share ~1.5 % (profiles/r04_s2/ab64*.log)
static bool dgemm_sub(GemmArgsT<double>& g, bool square_lower, hipStream_t st, hipError_t& e) {
  if (debug_inject_mask() & IPMZ_DEBUG_F64_ENGINE) return false;
  if (square_lower) {
    if (g.M <= IPMZ_TRAIL_SMALL_M) return false;
    return launch_dgemm_glds<128, 128, 4, 4, 8, 3, 8>(g, st, e);
  }
  if (g.M <= 4096) return launch_dgemm_glds<64, 64, 2, 2, 8, 3, 8, EPI_SUB_STRIP>(g, st, e);
  return launch_dgemm_glds<64, 128, 2, 2, 8, 3, 4, EPI_SUB_STRIP>(g, st, e);
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
  if constexpr (std::is_same<T, float>::value) {
    hipError_t e = hipSuccess;
    if (batch == 1 && sgemm_sub(g, square_lower, st, e)) return e;
  } else {
    hipError_t e = hipSuccess;
    if (batch == 1 && dgemm_sub(g, square_lower, st, e)) return e;
  }
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

// ---------------------------------------------------------------------------
// Factor the outer panel [k0, k0 + bo) as a kernel chain (batched factors
// and nbi = 128): inner diag / TRSM / strip steps, all on stream st.  Writes
// L (in K), D, the L11^{-1} blocks and W = L D for the panel's rows below
// each inner block (W: N x nbo, this panel's buffer).  Single-QP factors
// with nbi = 64 take the two-launch panel path of panel.hip instead.
template <typename T>
static hipError_t factor_panel(T* K, int64_t ld, int N, T* D, T* Linv, T* W, int k0, int bo, int nbo, int nbi,
                               int* info, hipStream_t st, const BatchStrides* bs = nullptr) {
  hipError_t e = hipSuccess;
  const int B = bs ? bs->B : 1;
  const int64_t sK = bs ? bs->sK : 0, sD = bs ? bs->sD : 0, sL = bs ? bs->sL : 0, sW = bs ? bs->sW : 0;
  for (int j0 = k0; j0 < k0 + bo; j0 += nbi) {
    const int bi = k0 + bo - j0 < nbi ? k0 + bo - j0 : nbi;
    T* Lb = Linv + (int64_t)(j0 / nbi) * nbi * nbi;
    if (nbi == 128)
      hipLaunchKernelGGL((ldlt_diag_kernel<T, 128>), dim3(B), dim3(1024), 0, st, K, ld, j0, bi, D, Lb, info, sK, sD, sL);
    else
      launch_diag64(B, st, K, ld, j0, bi, D, Lb, info, sK, sD, sL);
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
  if (nbi == 64 && N <= IPMZ_SMALL_NMAX) return ldlt_factor_small_batched(K, ld, N, D, Linv, W, info, st, bs);
  hipError_t e = hipSuccess;
  for (int k0 = 0; k0 < N; k0 += nbo) {
    const int bo = N - k0 < nbo ? N - k0 : nbo, t0 = k0 + bo;
    if ((e = factor_panel(K, ld, N, D, Linv, W, k0, bo, nbo, nbi, info, st, &bs)) != hipSuccess) return e;
    if (t0 < N && (e = panel_update(K, ld, N, W, nbo, k0, bo, t0, N, true, st, &bs)) != hipSuccess) return e;
  }
  return hipSuccess;
}

// Blocked LDL^T with depth-1 look-ahead.  With P_k the k-th outer panel
// (nbo columns), W_k = L_k D_k its rows below it (Ws: 3 buffers of N x nbo):
//
// Panel path of panel.hip (single QP, nbi = 64), THREE streams:
//   A (st, high priority): [wait N_{k-1}] the chain launch of P_{k+1}
//      (normally the diagonal-region roles, first updated with P_k; the
//      factor's critical path on ~nb CUs) -> event A_{k+1}
//   C (st3, high priority): [wait N_{k-1}, A_k] the look-ahead update of
//      P_{k+1}'s rows below its region with P_k (strip GEMM), then the rows
//      launch of P_{k+1}: their TRSMs / strips, pipelined behind the chain by
//      flags -> event C_{k+1};
//      A waits for it -> event P_{k+1} (the panel is complete)
//   The chain roles of a panel may run in either of its two launches
//   (panel.hip): C waits for A_k as well before panel k+1 reuses what panel
//   k's chain roles read (the pre-accumulated block (0, 0) slot).
//   B (st2, low priority): [wait P_k] update P_{k+2} with P_k -> event N_k;
//      the trailing update beyond P_{k+2} with P_k (the big GEMM, overlapping
//      the next panels)
// Kernel-chain path (batched / nbi = 128), two streams: A updates P_{k+1}
// with P_k (all rows) and factors it with factor_panel; B as above.
// Correctness: P_{k+1}'s columns get panel j <= k-1 contributions from B
// (ordered on B before N_{k-1}) and panel k's from A / C; B never touches the
// columns A / C factor; W is triple-buffered so panel k+1 never overwrites
// the W_{k-2} a late B_{k-2} could still read (B_{k-2} precedes N_{k-1}).
// A waits for B's tail at the end.
template <typename T>
static hipError_t ldlt_factor_t(T* K, int64_t ld, int N, T* D, T* Linv, T* W, int nbo, int nbi, int* info,
                                hipStream_t st, TrailTimer* timer, hipStream_t st2, hipStream_t st3, hipEvent_t* ev,
                                int nev, unsigned* pctrl, hipStream_t st4) {
  if (N <= 0) return hipSuccess;
  if (nbi != 64 && nbi != 128) return hipErrorInvalidValue;
  if (nbo % nbi != 0 || nbo > IPMZ_NBO_MAX) return hipErrorInvalidValue;
  const int npan = (N + nbo - 1) / nbo;
  const bool fused = pctrl != nullptr && nbi == 64;
  const bool two = st2 != nullptr && ev != nullptr && nev >= 4 * npan + 2 && (!fused || st3 != nullptr);
  // st4 (a fourth, high-priority stream): B's look-ahead strip beside the
  // trailing update instead of before it on B -- its short grid fills the
  // device's slots next to the trailing launch rather than running alone
  const bool four = two && st4 != nullptr && nev >= 5 * npan + 3 && !(debug_inject_mask() & IPMZ_DEBUG_NO_FOURTH);
  const int64_t wsz = (int64_t)N * nbo;
  auto Wb = [&](int k) { return W + (two ? (k % 3) : 0) * wsz; };  // T*
  auto pw = [&](int k) { return N - k * nbo < nbo ? N - k * nbo : nbo; };
  auto area = [&](int k) { return pctrl + (int64_t)IPMZ_PANEL_CTRL_WORDS * (1 + k); };
  unsigned* err = pctrl ? pctrl + PANEL_ERR_WORD : nullptr;
  hipStream_t sC = (two && fused) ? st3 : st;  // rows launches
  // early: panel k+1's chain launch does not wait for panel k's rows launch
  // (flags cover what it reads: RDONE).  It then holds its CUs beside that
  // launch's tail -- a gain where the panel chain is the critical path (small
  // N), a loss where the trailing GEMM is (it waits for that tail).  Never
  // inside a graph capture: a replay may run the two launches in either order
  // (no edge between them), and a chain launch spinning on a launch queued
  // behind it would only end at the spin limit.
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (two && fused && hipStreamIsCapturing(st, &cap) != hipSuccess) cap = hipStreamCaptureStatusActive;
  const bool early_ok = two && fused && cap == hipStreamCaptureStatusNone;
  // per panel j: its chain launch starts early once the order left from
  // its start is small enough (the chain-bound periods; C2 from its first
  // panel, C3 / C5 their last ones)
  auto early_at = [&](int j) { return early_ok && N - j * nbo <= IPMZ_EARLY_CHAIN_MAX_N; };
  // per panel j >= 1: the look-ahead update of its rows below the region as
  // strip tiles of its rows launch instead of a strip GEMM before it on C,
  // where the order left is as small (the chain-bound periods: the rows roles
  // then start as their own rows are done, not behind a whole GEMM launch, and
  // keep pace with the chain; panel.hip strip_tile).  Capture or not alike, so
  // a captured step computes what an eager one does.
  auto tiles_at = [&](int j) { return two && fused && N - j * nbo <= IPMZ_EARLY_CHAIN_MAX_N; };
  // per panel j >= 2 whose previous panel was early too: the B stream's
  // look-ahead update of its columns (N_{j-2}) reaches its chain launch as a
  // flag (panel_ready after that update on B; the chain roles poll it and
  // acquire) instead of a cross-stream wait on A -- each such wait costs a
  // launch several us even when already satisfied.  N_{j-2} also stands for
  // the rows launch of panel j - 2 (B waited for it) and so for the W buffer
  // the panel reuses.  The rows launch keeps its wait on C: its hundreds of
  // workgroups spinning on the flag could hold every CU the B stream's
  // update needs (the chain launch's few dozen cannot).
  auto flag_at = [&](int j) { return j >= 2 && early_at(j - 1) && tiles_at(j); };
  // the next panel's block (0, 0) look-ahead update, pre-accumulated by the
  // rows launch of panel k into slot (k + 1) % 3 (after the ctrl areas): the
  // rows launch of panel k + 1 reuses the slot that panel k - 1's chain roles
  // read, before panel k's chain started (so C need not wait for A_k)
  T* pre00 = pctrl ? reinterpret_cast<T*>(pctrl + (int64_t)IPMZ_PANEL_CTRL_WORDS * (1 + npan)) : nullptr;
  auto slot00 = [&](int k) { return pre00 + (int64_t)(k % 3) * 64 * 64; };
  auto factor = [&](int k, bool prev) -> hipError_t {  // panel k (prev: with the look-ahead update from k - 1)
    const int k0 = k * nbo;
    if (!fused) return factor_panel(K, ld, N, D, Linv, Wb(k), k0, pw(k), nbo, nbi, info, st);
    return panel_factor(K, ld, N, k0, pw(k), D, Linv + (int64_t)(k0 / 64) * 64 * 64, Wb(k), nbo,
                        (two && prev) ? slot00(k) : nullptr, two ? slot00(k + 1) : nullptr, info, area(k), err,
                        prev ? Wb(k - 1) : nullptr, k0 - nbo, nbo, prev && tiles_at(k), st, sC,
                        (early_at(k) && prev) ? area(k - 1) : nullptr, prev && flag_at(k));
  };
  hipError_t e = hipSuccess;
  if (!two) {  // single stream: factor, then the whole trailing update
    for (int k = 0; k < npan; ++k) {
      const int k0 = k * nbo, bo = pw(k), t0 = k0 + bo;
      if ((e = factor(k, false)) != hipSuccess) return e;
      if (t0 < N) {
        // timed: the launches of the dominant 128 x 128 trailing kernel
        hipEvent_t* te = timer && N - t0 > IPMZ_TRAIL_SMALL_M ? timer->next() : nullptr;
        if (te) hipEventRecord(te[0], st);
        e = panel_update(K, ld, N, Wb(k), nbo, k0, bo, t0, N, true, st);
        if (te) hipEventRecord(te[1], st);
        if (te) timer->flops += (double)(N - t0) * (double)(N - t0 + 1) * (double)bo;
        if (e != hipSuccess) return e;
      }
    }
    return hipSuccess;
  }
  hipEvent_t* evP = ev;             // panel k complete (A)
  hipEvent_t* evN = ev + npan;      // P_{k+2} updated with P_k (B)
  hipEvent_t* evC = ev + 2 * npan;  // rows launch of panel k done (C)
  hipEvent_t* evA = ev + 3 * npan;  // chain launch of panel k done (A)
  hipEvent_t* evT = ev + 4 * npan + 2;  // trailing update with panel k done (B; four streams)
  hipEvent_t evJoin = ev[4 * npan];
  hipEvent_t evJoin4 = four ? ev[5 * npan + 2] : nullptr;
  // everything the caller enqueued on st before the factor (the mixed path's
  // fp32 conversion, the ctrl-word memsets) comes first on B and C as well
  hipEvent_t evEntry = ev[4 * npan + 1];
  IPMZ_TRACE("factor: N=%d npan=%d look-ahead", N, npan);
  if ((e = stream_record(evEntry, st)) != hipSuccess) return e;
  if ((e = stream_wait(st2, evEntry)) != hipSuccess) return e;
  if (fused && (e = stream_wait(sC, evEntry)) != hipSuccess) return e;
  if ((e = factor(0, false)) != hipSuccess) return e;
  if (fused) {
    if ((e = stream_record(evA[0], st)) != hipSuccess) return e;
    if ((e = stream_record(evC[0], sC)) != hipSuccess) return e;
    if (!early_at(1) && (e = stream_wait(st, evC[0])) != hipSuccess) return e;
  }
  for (int k = 0; k < npan; ++k) {
    const int k0 = k * nbo, bo = pw(k);
    const int p1 = k0 + bo;                          // start of P_{k+1}
    const int p2 = p1 < N ? p1 + pw(k + 1) : N;      // start of P_{k+2}
    const int p3 = p2 < N ? p2 + pw(k + 2) : N;      // start of P_{k+3}
    if (p1 >= N) break;
    IPMZ_TRACE("factor: panel %d", k);
    if ((e = stream_record(evP[k], st)) != hipSuccess) return e;
    // ---- stream B: P_{k+2} columns first, then the rest (four streams: the
    // P_{k+2} strip on st4 after B's previous trailing update, which last
    // touched those columns; B goes straight on with the rest)
    // (early: panel k's rows launch on C as well -- A no longer waits for it)
    if ((e = stream_wait(st2, evP[k])) != hipSuccess) return e;
    if (early_at(k + 1) && (e = stream_wait(st2, evC[k])) != hipSuccess) return e;
    hipStream_t sN = four ? st4 : st2;  // the stream of the P_{k+2} strip and N_k
    if (four) {
      if ((e = stream_wait(st4, evP[k])) != hipSuccess) return e;
      if (early_at(k + 1) && (e = stream_wait(st4, evC[k])) != hipSuccess) return e;
      if (k >= 1 && (e = stream_wait(st4, evT[k - 1])) != hipSuccess) return e;
    }
    if (p2 < N) {
      if ((e = panel_update(K, ld, N, Wb(k), nbo, k0, bo, p2, p3, false, sN)) != hipSuccess) return e;
      if (k + 2 < npan && flag_at(k + 2) && (e = panel_ready(area(k + 2), sN)) != hipSuccess) return e;
    }
    if ((e = stream_record(evN[k], sN)) != hipSuccess) return e;
    if (p3 < N) {
      hipEvent_t* te = timer && N - p3 > IPMZ_TRAIL_SMALL_M ? timer->next() : nullptr;
      if (te) hipEventRecord(te[0], st2);
      e = panel_update(K, ld, N, Wb(k), nbo, k0, bo, p3, N, true, st2);
      if (te) hipEventRecord(te[1], st2);
      if (te) timer->flops += (double)(N - p3) * (double)(N - p3 + 1) * (double)bo;
      if (e != hipSuccess) return e;
    }
    if (four && (e = stream_record(evT[k], st2)) != hipSuccess) return e;
    // ---- streams A (and C): update P_{k+1} with P_k, factor P_{k+1}
    if (k >= 1) {
      if (!flag_at(k + 1) && (e = stream_wait(st, evN[k - 1])) != hipSuccess) return e;
      if (fused && (e = stream_wait(sC, evN[k - 1])) != hipSuccess) return e;
    }
    if (k >= 1) {
      // early: panel k-1's rows launch (and C's strip before it) are the last
      // readers of W buffer (k + 1) % 3 -- the one this chain launch writes.
      // Where panel k was early too, B waited for that launch before N_{k-1}
      // (above), so the wait on N_{k-1} covers it: one cross-stream wait
      // fewer before the chain launch (each costs the launch several us)
      if (early_at(k + 1) && !early_at(k) && (e = stream_wait(st, evC[k - 1])) != hipSuccess) return e;
    }
    if (fused) {
      // the look-ahead update with P_k: the rows below P_{k+1}'s diagonal
      // region as a strip GEMM on C (beside the chain launch, which updates
      // the region itself); panel k's chain roles may have run in its chain
      // launch, so C also waits for that launch -- except with strip tiles:
      // then the rows launch reads nothing the chain launch of panel k writes
      // but through flags, and the block (0, 0) slot it reuses was read
      // before panel k's chain started (three slots)
      if (!tiles_at(k + 1) && (e = stream_wait(sC, evA[k])) != hipSuccess) return e;
      if (p2 < N && !tiles_at(k + 1)) {
        if ((e = gemm_nt_sub_t<T>(N - p2, p2 - p1, bo, Wb(k) + (int64_t)p2 * nbo, nbo, K + (int64_t)p1 * ld + k0, ld,
                                  K + (int64_t)p2 * ld + p1, ld, p2, p1, false, sC, nullptr)) != hipSuccess)
          return e;
      }
      if ((e = factor(k + 1, true)) != hipSuccess) return e;
      if ((e = stream_record(evA[k + 1], st)) != hipSuccess) return e;
      if ((e = stream_record(evC[k + 1], sC)) != hipSuccess) return e;
      if (!early_at(k + 2) && (e = stream_wait(st, evC[k + 1])) != hipSuccess) return e;
    } else {
      if ((e = panel_update(K, ld, N, Wb(k), nbo, k0, bo, p1, p2, false, st)) != hipSuccess) return e;
      if ((e = factor(k + 1, false)) != hipSuccess) return e;
    }
  }
  if (early_ok && (e = stream_wait(st, evC[npan - 1])) != hipSuccess) return e;  // the last rows launch
  if ((e = stream_record(evJoin, st2)) != hipSuccess) return e;
  if (four) {
    if ((e = stream_record(evJoin4, st4)) != hipSuccess) return e;
    if ((e = stream_wait(st, evJoin4)) != hipSuccess) return e;
  }
  return stream_wait(st, evJoin);
}

hipError_t ldlt_factor(double* K, int64_t ld, int N, double* D, double* Linv, double* W, int nbo, int nbi,
                       int* info, hipStream_t st, TrailTimer* timer, hipStream_t st2, hipStream_t st3, hipEvent_t* ev,
                       int nev, unsigned* pctrl, hipStream_t st4) {
  return ldlt_factor_t<double>(K, ld, N, D, Linv, W, nbo, nbi, info, st, timer, st2, st3, ev, nev, pctrl, st4);
}
hipError_t ldlt_factor(float* K, int64_t ld, int N, float* D, float* Linv, float* W, int nbo, int nbi, int* info,
                       hipStream_t st, TrailTimer* timer, hipStream_t st2, hipStream_t st3, hipEvent_t* ev, int nev,
                       unsigned* pctrl, hipStream_t st4) {
  return ldlt_factor_t<float>(K, ld, N, D, Linv, W, nbo, nbi, info, st, timer, st2, st3, ev, nev, pctrl, st4);
}

}  // namespace ipmz
