// NT GEMM tile engine of the factorization (trailing and strip updates, the
// panel TRSM of the kernel-chain path): templates shared by ldlt.hip and the
// kbench experiment tool (tools/kbench_probes.hip).
#pragma once
#include "common.h"

namespace ipmz {

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
  int persist;  // OPT_PERSIST: grid size (0: one workgroup per tile)
  // batch (blockIdx.y = QP): element strides between the QPs' operands
  int64_t sA, sB, sC, sW, sD;
};
using GemmArgs = GemmArgsT<double>;

// Tile pipeline: one LDS buffer is computed while the next k-chunk sits in
// registers (loads issued before the MFMAs, written to the other buffer
// after them): one barrier per 16-deep k-chunk.
template <typename T, int BM, int BN, int NTH, int BK_ = 16>
struct TileLoader {
  typedef typename Mfma<T>::vec2_t V2;
  static constexpr int BK = BK_, PAD = BK_ + 2;  // (PAD = BK + 2: conflict-free fragment reads for BK 16 and 32)
  static constexpr int CPR = BK / 2;             // double2 / float2 chunks per row
  static constexpr int QA = BM * BK / 2 / NTH, QB = BN * BK / 2 / NTH;  // double2 per thread
  // every thread loads whole double2 chunks: a tile side with fewer chunks
  // than threads (e.g. BM = 64 at 16 waves) would load NOTHING
  static_assert(QA * NTH * 2 == BM * BK && QB * NTH * 2 == BN * BK, "tile side too small for this wave grid");
  V2 ra[QA], rb[QB];
  __device__ __forceinline__ void load(const GemmArgsT<T>& g, int i0, int j0, int kk) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int ch = tid + NTH * q, r = ch / CPR, c = (ch % CPR) * 2;
      ra[q] = fetch(g.A, g.lda, i0 + r, g.M, kk + c, g.Kd);
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int ch = tid + NTH * q, r = ch / CPR, c = (ch % CPR) * 2;
      rb[q] = fetch(g.B, g.ldb, j0 + r, g.N, kk + c, g.Kd);
    }
  }
  __device__ __forceinline__ void store(T* As, T* Bs) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int ch = tid + NTH * q, r = ch / CPR, c = (ch % CPR) * 2;
      *reinterpret_cast<V2*>(&As[r * PAD + c]) = ra[q];
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int ch = tid + NTH * q, r = ch / CPR, c = (ch % CPR) * 2;
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
//   OPT_PERSIST  a bounded grid (GemmArgs::persist workgroups) that loops over
//             the tiles: the launch never holds every CU slot, so panel
//             workgroups launched beside it are dispatched at once instead of
//             waiting for the whole GEMM to drain
enum { OPT_NOR2 = 2, OPT_GRP = 4, OPT_PERSIST = 8 };
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

// Tiles are sized for two workgroups per CU: 8 waves = 4 per SIMD (<= 128
// VGPRs), 16 waves = 8 per SIMD (<= 64 VGPRs).  Pinned with
// amdgpu_waves_per_eu: the compiler otherwise drifts past the budget and
// silently halves the occupancy.
template <int NW>
constexpr int gemm_waves_per_eu() { return NW == 16 ? 8 : NW == 8 ? 4 : 1; }
// BK: k-depth of one LDS stage (one barrier per stage)
template <typename T, int BM, int BN, int EPI, int WGM = 2, int WGN = 2, int OPT = OPT_NOR2, int BK = 16>
__global__ __launch_bounds__(64 * WGM * WGN)
__attribute__((amdgpu_waves_per_eu(gemm_waves_per_eu<WGM * WGN>()))) void gemm_nt_kernel(GemmArgsT<T> g) {
  typedef Mfma<T> MF;
  constexpr int PAD = BK + 2, NTH = 64 * WGM * WGN;
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
  int bid0 = blockIdx.x;
  {
    const int nwg = gridDim.x, q = nwg / 8, r = nwg % 8, x = bid0 % 8;
    bid0 = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid0 / 8;
  }
  const int ntiles = (OPT & OPT_PERSIST) ? (g.lower == 2 ? g.ntm * (g.ntm + 1) / 2 : g.ntm * g.ntn) : bid0 + 1;
  for (int bid = bid0; bid < ntiles; bid += gridDim.x) {
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
  if (g.lower == 1 && g.row0 + i0 + BM - 1 < g.col0 + j0) continue;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WGN, wc = wave % WGN;
  typename MF::acc_t acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = (typename MF::acc_t){T(0), T(0), T(0), T(0)};

  TileLoader<T, BM, BN, NTH, BK> ld;
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
  }  // tiles
}

template <int BM, int BN, int EPI, int WGM = 2, int WGN = 2, int OPT = OPT_NOR2, int BK = 16, typename T = double>
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
  if ((OPT & OPT_PERSIST) && g.persist > 0 && nblk > g.persist) nblk = g.persist;
  hipLaunchKernelGGL((gemm_nt_kernel<T, BM, BN, EPI, WGM, WGN, OPT, BK>), dim3((unsigned)nblk, (unsigned)batch),
                     dim3(64 * WGM * WGN), 0, st, g);
  return hipGetLastError();
}

}  // namespace ipmz
