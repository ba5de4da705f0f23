// fp32 NT GEMM of the mixed-precision factor (C5): the trailing update
// C -= W L^T of the fp32 LDL^T (LinearSolvers.cpp:30-36 in fp32, rank nbo)
// and its look-ahead strips, on v_mfma_f32_32x32x2_f32.
//
// Why a kernel of its own: the shared engine (gemm.h) is built around the
// 16 x 16 x 4 shape of the f64 MFMA.  Its fp32 instance reads one float per
// lane per 16 x 16 x 4 MFMA from LDS (ds_read_b32, 32 cycles of MFMA per
// read pair) and ran at 89 TFLOP/s alone at R = 15872, rank 512
// (profiles/r03_s3/gemmref32.log).  Here:
//   * 32 x 32 x 2 f32 MFMA (64 cycles each, 16 accumulators per lane): a wave
//     tile of TM x TN 32 x 32 blocks;
//   * each lane reads FOUR consecutive k of its row with one ds_read_b128 and
//     feeds them to four MFMAs (MFMA s of a group of 8 k takes k = 4 h + s,
//     h = lane >> 5, on both operands): 2 (TM + TN) b128 reads per 4 TM TN
//     MFMAs;
//   * LDS rows padded to BK + 4 floats (an odd number of 16-byte slots), so
//     the 16 rows of each ds_read_b128 lane group hit 16 distinct slots;
//   * the next k-chunk's global loads (float4, row-contiguous) are issued
//     before the current chunk's MFMAs and written to the other LDS buffer
//     after them: one barrier per chunk;
//   * the tile order of gemm.h (XCD-aware remap, grouped triangular
//     enumeration for the trailing triangle).
// The MFMA result is an exact f32 fma chain in a fixed k order, so a launch
// is deterministic (eager and captured steps run the same code).
//
// C/D layout of the 32 x 32 MFMAs (cdna_hip_programming.md §3): column
// lane & 31, row (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5).
#pragma once
#include "common.h"
#include "gemm.h"

namespace ipmz {

typedef float float16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float16_t mfma_f32_32x32x2(float a, float b, float16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

template <int BM, int BN, int NTH, int BK>
struct Loader32 {
  static constexpr int PADK = BK + 4;
  static constexpr int CPR = BK / 4;  // float4 chunks per row
  static constexpr int QA = BM * BK / 4 / NTH, QB = BN * BK / 4 / NTH;
  static_assert(QA * NTH * 4 == BM * BK && QB * NTH * 4 == BN * BK, "tile side too small for this workgroup");
  float4 ra[QA], rb[QB];
  static __device__ __forceinline__ float4 fetch(const float* P, int64_t ld, int row, int rows, int k, int Kd) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < rows) {
      const float* p = P + (int64_t)row * ld + k;
      if (k + 3 < Kd) {
        t = *reinterpret_cast<const float4*>(p);
      } else {
        if (k < Kd) t.x = p[0];
        if (k + 1 < Kd) t.y = p[1];
        if (k + 2 < Kd) t.z = p[2];
      }
    }
    return t;
  }
  __device__ __forceinline__ void load(const GemmArgsT<float>& g, int i0, int j0, int kk) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int ch = tid + NTH * q, r = ch / CPR, c = (ch % CPR) * 4;
      ra[q] = fetch(g.A, g.lda, i0 + r, g.M, kk + c, g.Kd);
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int ch = tid + NTH * q, r = ch / CPR, c = (ch % CPR) * 4;
      rb[q] = fetch(g.B, g.ldb, j0 + r, g.N, kk + c, g.Kd);
    }
  }
  __device__ __forceinline__ void store(float* As, float* Bs) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int ch = tid + NTH * q, r = ch / CPR, c = (ch % CPR) * 4;
      *reinterpret_cast<float4*>(&As[r * PADK + c]) = ra[q];
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int ch = tid + NTH * q, r = ch / CPR, c = (ch % CPR) * 4;
      *reinterpret_cast<float4*>(&Bs[r * PADK + c]) = rb[q];
    }
  }
};

// WPE: waves per SIMD the tile is built for (register budget 512 / WPE);
// EPI: EPI_SUB (trailing triangle) or EPI_SUB_STRIP (look-ahead strip) -- the
// same code, separate instantiations so kernel traces tell them apart
template <int BM, int BN, int WGM, int WGN, int BK, int WPE, int EPI = EPI_SUB>
__global__ __launch_bounds__(64 * WGM * WGN) __attribute__((amdgpu_waves_per_eu(WPE))) void sgemm_nt_kernel(
    GemmArgsT<float> g) {
  constexpr int NTH = 64 * WGM * WGN, WM = BM / WGM, WN = BN / WGN, TM = WM / 32, TN = WN / 32;
  constexpr int PADK = BK + 4;
  static_assert(WM % 32 == 0 && WN % 32 == 0 && BK % 8 == 0, "32 x 32 blocks, k groups of 8");
  if (blockIdx.y) {
    const int64_t z = blockIdx.y;
    g.A += z * g.sA;
    g.B += z * g.sB;
    g.C += z * g.sC;
  }
  __shared__ __attribute__((aligned(16))) float As[2][BM * PADK];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * PADK];

  int bid = blockIdx.x;
  {  // XCD-aware remap (bijective), as gemm.h
    const int nwg = gridDim.x, q = nwg / 8, r = nwg % 8, x = bid % 8;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  int tm, tn;
  if (g.lower == 2) {
    grouped_tile(bid, g.ntm, tm, tn);
  } else {
    tn = bid % g.ntn;
    tm = bid / g.ntn;
  }
  const int i0 = tm * BM, j0 = tn * BN;
  if (g.lower == 1 && g.row0 + i0 + BM - 1 < g.col0 + j0) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WGN, wc = wave % WGN;

  float16_t acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  Loader32<BM, BN, NTH, BK> ld;
  const int nch = (g.Kd + BK - 1) / BK;
  ld.load(g, i0, j0, 0);
  ld.store(As[0], Bs[0]);
  __syncthreads();
  // lane l reads row (l & 31) of its 32-row block, k = 4 (l >> 5) .. + 3 of a group of 8
  const int aoff = (wr * WM + (lane & 31)) * PADK + 4 * (lane >> 5);
  const int boff = (wc * WN + (lane & 31)) * PADK + 4 * (lane >> 5);
  for (int t = 0; t < nch; ++t) {
    const int cur = t & 1;
    if (t + 1 < nch) ld.load(g, i0, j0, (t + 1) * BK);
    const float* as = As[cur];
    const float* bs = Bs[cur];
#pragma unroll
    for (int q = 0; q < BK / 8; ++q) {
      float4 af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = *reinterpret_cast<const float4*>(&as[aoff + a * 32 * PADK + 8 * q]);
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b] = *reinterpret_cast<const float4*>(&bs[boff + b * 32 * PADK + 8 * q]);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          acc[a][b] = mfma_f32_32x32x2(af[a].x, bf[b].x, acc[a][b]);
          acc[a][b] = mfma_f32_32x32x2(af[a].y, bf[b].y, acc[a][b]);
          acc[a][b] = mfma_f32_32x32x2(af[a].z, bf[b].z, acc[a][b]);
          acc[a][b] = mfma_f32_32x32x2(af[a].w, bf[b].w, acc[a][b]);
        }
    }
    if (t + 1 < nch) ld.store(As[cur ^ 1], Bs[cur ^ 1]);
    __syncthreads();
  }

  // epilogue: C -= acc (a row of 32 consecutive columns per register)
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int j = j0 + wc * WN + b * 32 + (lane & 31);
      if (j >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + wr * WM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (i < g.M) {
          float* cp = g.C + (int64_t)i * g.ldc + j;
          *cp = *cp - acc[a][b][r];
        }
      }
    }
}

// the operands' float4 loads need 16-byte aligned rows
inline bool sgemm_aligned(const GemmArgsT<float>& g) {
  return ((reinterpret_cast<uintptr_t>(g.A) | reinterpret_cast<uintptr_t>(g.B)) & 15) == 0 && g.lda % 4 == 0 &&
         g.ldb % 4 == 0 && (g.sA % 4) == 0 && (g.sB % 4) == 0;
}

template <int BM, int BN, int WGM, int WGN, int BK, int WPE, int EPI = EPI_SUB>
static hipError_t launch_sgemm(GemmArgsT<float> g, hipStream_t st, int batch = 1) {
  g.ntm = (g.M + BM - 1) / BM;
  g.ntn = (g.N + BN - 1) / BN;
  if (g.ntm == 0 || g.ntn == 0 || g.Kd == 0) return hipSuccess;
  if (!sgemm_aligned(g)) return hipErrorInvalidValue;
  int64_t nblk = (int64_t)g.ntm * g.ntn;
  if (g.lower == 2) {
    if (BM == BN) nblk = (int64_t)g.ntm * (g.ntm + 1) / 2;
    else g.lower = 1;
  }
  hipLaunchKernelGGL((sgemm_nt_kernel<BM, BN, WGM, WGN, BK, WPE, EPI>), dim3((unsigned)nblk, (unsigned)batch),
                     dim3(64 * WGM * WGN), 0, st, g);
  return hipGetLastError();
}

}  // namespace ipmz
