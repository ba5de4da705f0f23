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
typedef float f32x4 __attribute__((ext_vector_type(4)));

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
  // FULL: the tile lies inside the operands and Kd % BK == 0 (no per-element
  // predicates: unconditional loads the compiler can batch)
  template <bool FULL>
  static __device__ __forceinline__ float4 fetch(const float* P, int64_t ld, int row, int rows, int k, int Kd) {
    if constexpr (FULL) return *reinterpret_cast<const float4*>(P + (int64_t)row * ld + k);
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
  template <bool FULL>
  __device__ __forceinline__ void load(const GemmArgsT<float>& g, int i0, int j0, int kk) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int ch = tid + NTH * q, r = ch / CPR, c = (ch % CPR) * 4;
      ra[q] = fetch<FULL>(g.A, g.lda, i0 + r, g.M, kk + c, g.Kd);
    }
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int ch = tid + NTH * q, r = ch / CPR, c = (ch % CPR) * 4;
      rb[q] = fetch<FULL>(g.B, g.ldb, j0 + r, g.N, kk + c, g.Kd);
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

// The k loop of one output tile: acc (TM x TN 32 x 32 blocks of this wave)
template <int BM, int BN, int WGM, int WGN, int BK, bool FULL, int TM, int TN>
__device__ __forceinline__ void sgemm_tile_loop(const GemmArgsT<float>& g, int i0, int j0, float* As0, float* Bs0,
                                                float16_t (&acc)[TM][TN]) {
  constexpr int NTH = 64 * WGM * WGN, WM = BM / WGM, WN = BN / WGN;
  constexpr int PADK = BK + 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WGN, wc = wave % WGN;
  Loader32<BM, BN, NTH, BK> ld;
  const int nch = (g.Kd + BK - 1) / BK;
  ld.template load<FULL>(g, i0, j0, 0);
  ld.store(As0, Bs0);
  __syncthreads();
  // lane l reads row (l & 31) of its 32-row block, k = 4 (l >> 5) .. + 3 of a group of 8
  const int aoff = (wr * WM + (lane & 31)) * PADK + 4 * (lane >> 5);
  const int boff = (wc * WN + (lane & 31)) * PADK + 4 * (lane >> 5);
  for (int t = 0; t < nch; ++t) {
    const int cur = t & 1;
    if (t + 1 < nch) ld.template load<FULL>(g, i0, j0, (t + 1) * BK);
    const float* as = As0 + cur * BM * PADK;
    const float* bs = Bs0 + cur * BN * PADK;
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
    if (t + 1 < nch) ld.store(As0 + (cur ^ 1) * BM * PADK, Bs0 + (cur ^ 1) * BN * PADK);
    __syncthreads();
  }
}

// WPE: waves per SIMD the tile is built for (register budget 512 / WPE);
// EPI: EPI_SUB (trailing triangle) or EPI_SUB_STRIP (look-ahead strip) -- the
// same code, separate instantiations so kernel traces tell them apart
template <int BM, int BN, int WGM, int WGN, int BK, int WPE, int EPI = EPI_SUB>
__global__ __launch_bounds__(64 * WGM * WGN) __attribute__((amdgpu_waves_per_eu(WPE))) void sgemm_nt_kernel(
    GemmArgsT<float> g) {
  constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 32, TN = WN / 32;
  constexpr int PADK = BK + 4;
  static_assert(WM % 32 == 0 && WN % 32 == 0 && BK % 8 == 0, "32 x 32 blocks, k groups of 8");
  if (blockIdx.y) {
    const int64_t z = blockIdx.y;
    g.A += z * g.sA;
    g.B += z * g.sB;
    g.C += z * g.sC;
  }
  __shared__ __attribute__((aligned(16))) float As[2 * BM * PADK];
  __shared__ __attribute__((aligned(16))) float Bs[2 * BN * PADK];

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
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WGN, wc = wave % WGN;

  float16_t acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  if (i0 + BM <= g.M && j0 + BN <= g.N && g.Kd % BK == 0)
    sgemm_tile_loop<BM, BN, WGM, WGN, BK, true>(g, i0, j0, As, Bs, acc);
  else
    sgemm_tile_loop<BM, BN, WGM, WGN, BK, false>(g, i0, j0, As, Bs, acc);

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

// ---------------------------------------------------------------------------
// The same tile with the operands staged by LDS-DMA (global_load_lds_dwordx4:
// no VGPR staging, no ds_write pass) through an NST-deep LDS ring: stage t+2
// is in flight while stage t is computed (counted vmcnt + raw s_barrier, so
// the DMA of the next stages stays in flight across the barrier).
// LDS image of one stage: [rows][BK floats] unpadded, the 16-byte slots of a
// row XOR-swizzled (slot c of row r at c ^ f(r), f(r) = (r / (16 / SLOTS)) %
// SLOTS, SLOTS = BK / 4): a DMA wave-instruction writes 1 KB lane-linearly, so
// the swizzle is applied to each lane's SOURCE address, and the 16 rows of
// each ds_read_b128 lane group land on 16 distinct bank slots.
// Full tiles only (i0 + BM <= M, j0 + BN <= N, Kd % BK == 0): the caller
// routes the rest to sgemm_tile_loop.
// s_waitcnt immediate (gfx9 encoding): vmcnt(n), lgkmcnt(0), expcnt untouched
constexpr int vmcnt_lgkm0(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4); }
template <int BK>
__device__ __forceinline__ int glds_swz(int r) {
  constexpr int SLOTS = BK / 4, RPB = 16 / SLOTS;  // 16-byte slots per row, rows per 256-byte bank row
  return (r / RPB) % SLOTS;
}
__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)p;
}
template <int BM, int BN, int WGM, int WGN, int BK, int NST, bool RDA, int TM, int TN>
__device__ __forceinline__ void sgemm_tile_loop_glds(const GemmArgsT<float>& g, int i0, int j0, float* ring0,
                                                     float* ring1, float* ring2, float16_t (&acc)[TM][TN]) {
  constexpr int NW = WGM * WGN, WM = BM / WGM, WN = BN / WGN;
  constexpr int SLOTS = BK / 4, RPI = 64 / SLOTS;          // rows per DMA wave-instruction
  constexpr int IA = BM / RPI, IB = BN / RPI;              // DMA instructions per stage
  static_assert((IA + IB) % NW == 0, "DMA instructions split evenly over the waves");
  constexpr int LPW = (IA + IB) / NW;                      // per wave per stage
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / WGN, wc = wave % WGN;
  const int nch = g.Kd / BK;
  // this lane's DMA sources: instruction m of the stage (m = wave + NW * u)
  const int rl = lane / SLOTS, phys = lane % SLOTS;
  // stage t lives in ring buffer t % NST; the k loop is unrolled by NST so
  // every buffer offset is a compile-time constant (hipcc then sees that the
  // DMA into one buffer cannot alias the ds_reads of another and emits no
  // vmcnt(0) before them)
  auto ring = [&](auto bc) -> float* {
    constexpr int B = decltype(bc)::value;
    if constexpr (B == 0) return ring0;
    else if constexpr (B == 1) return ring1;
    else return ring2;
  };
  auto issue = [&](int t, auto bc) {
    float* st = ring(bc);
    const int kk = t * BK;
#pragma unroll
    for (int u = 0; u < LPW; ++u) {
      const int m = wave + NW * u;
      const float* src;
      float* dst;
      if (m < IA) {
        const int r = m * RPI + rl;
        src = g.A + (int64_t)(i0 + r) * g.lda + kk + 4 * (phys ^ glds_swz<BK>(r));
        dst = st + m * 256;
      } else {
        const int r = (m - IA) * RPI + rl;
        src = g.B + (int64_t)(j0 + r) * g.ldb + kk + 4 * (phys ^ glds_swz<BK>(r));
        dst = st + BM * BK + (m - IA) * 256;
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };
  // one 8-deep k group: the fragments of this wave (lane l: row l & 31 of
  // each 32-row block, k = 4 (l >> 5) .. + 3) and its 4 TM TN MFMAs
  auto rd_asm = [&](const float* as, const float* bs, int q, f32x4 (&af)[TM], f32x4 (&bf)[TN]) {
    const int c = 2 * q + (lane >> 5);
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int r = wr * WM + a * 32 + (lane & 31);
      asm volatile("ds_read_b128 %0, %1" : "=v"(af[a]) : "v"(lds_addr(&as[r * BK + 4 * (c ^ glds_swz<BK>(r))])) : "memory");
    }
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int r = wc * WN + b * 32 + (lane & 31);
      asm volatile("ds_read_b128 %0, %1" : "=v"(bf[b]) : "v"(lds_addr(&bs[r * BK + 4 * (c ^ glds_swz<BK>(r))])) : "memory");
    }
  };
  // wait for the asm reads in flight; the MFMAs issued so far stay before the
  // wait (their accumulators tied to it), the fragments' uses after it
  auto wait_rd = [&](f32x4 (&af)[TM], f32x4 (&bf)[TN]) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) asm volatile("" : "+v"(acc[a][b]));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int a = 0; a < TM; ++a) asm volatile("" : "+v"(af[a]));
#pragma unroll
    for (int b = 0; b < TN; ++b) asm volatile("" : "+v"(bf[b]));
  };
  auto mm = [&](const f32x4 (&af)[TM], const f32x4 (&bf)[TN]) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        acc[a][b] = mfma_f32_32x32x2(af[a][0], bf[b][0], acc[a][b]);
        acc[a][b] = mfma_f32_32x32x2(af[a][1], bf[b][1], acc[a][b]);
        acc[a][b] = mfma_f32_32x32x2(af[a][2], bf[b][2], acc[a][b]);
        acc[a][b] = mfma_f32_32x32x2(af[a][3], bf[b][3], acc[a][b]);
      }
  };
  auto compute = [&](auto bc) {
    const float* as = ring(bc);
    const float* bs = as + BM * BK;
    if constexpr (RDA) {
      // ds_read_b128 in asm (invisible to hipcc's wait insertion, which
      // otherwise drains every LDS-DMA in flight before the first read of a
      // pass over the ring), waited for by hand; group q + 1's reads are in
      // flight during group q's MFMAs
      f32x4 af0[TM], bf0[TN], af1[TM], bf1[TN];
      rd_asm(as, bs, 0, af0, bf0);
      wait_rd(af0, bf0);
#pragma unroll
      for (int q = 0; q < BK / 8; ++q) {
        const bool more = q + 1 < BK / 8;
        if (q & 1) {
          if (more) rd_asm(as, bs, q + 1, af0, bf0);
          mm(af1, bf1);
          if (more) wait_rd(af0, bf0);
        } else {
          if (more) rd_asm(as, bs, q + 1, af1, bf1);
          mm(af0, bf0);
          if (more) wait_rd(af1, bf1);
        }
      }
    } else {
#pragma unroll
      for (int q = 0; q < BK / 8; ++q) {
        f32x4 af[TM], bf[TN];
        const int c = 2 * q + (lane >> 5);
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          const int r = wr * WM + a * 32 + (lane & 31);
          af[a] = *reinterpret_cast<const f32x4*>(&as[r * BK + 4 * (c ^ glds_swz<BK>(r))]);
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int r = wc * WN + b * 32 + (lane & 31);
          bf[b] = *reinterpret_cast<const f32x4*>(&bs[r * BK + 4 * (c ^ glds_swz<BK>(r))]);
        }
        mm(af, bf);
      }
    }
  };
  // (the waits as s_waitcnt builtins, not asm: hipcc's wait insertion then
  // knows stage t's DMA has landed; the steady loop has no data-dependent
  // branch, so it adds no vmcnt(0) of its own before the ds_reads)
  static_for<NST - 1>([&](auto sc) {
    if (decltype(sc)::value < nch) issue(decltype(sc)::value, sc);
  });
  int t0 = 0;
  // steady state: every stage issued here exists (t0 + 2 (NST - 1) < nch)
  for (; t0 + 2 * (NST - 1) < nch; t0 += NST) {
    static_for<NST>([&](auto sc) {
      constexpr int S = decltype(sc)::value;
      __builtin_amdgcn_s_waitcnt(vmcnt_lgkm0((NST - 2) * LPW));  // stage t0 + S landed, later ones in flight
      __builtin_amdgcn_s_barrier();
      issue(t0 + S + NST - 1, std::integral_constant<int, (S + NST - 1) % NST>{});  // stage t - 1's buffer: read by all
      compute(sc);
    });
  }
  // tail: the last stages, waits counted down
  static_for<2 * NST - 1>([&](auto uc) {
    constexpr int U = decltype(uc)::value, S = U % NST;
    const int t = t0 + U;
    if (t < nch) {
      if (t + 1 < nch && NST == 3) __builtin_amdgcn_s_waitcnt(vmcnt_lgkm0(LPW));
      else __builtin_amdgcn_s_waitcnt(vmcnt_lgkm0(0));
      __builtin_amdgcn_s_barrier();
      if (t + NST - 1 < nch) issue(t + NST - 1, std::integral_constant<int, (S + NST - 1) % NST>{});
      compute(std::integral_constant<int, S>{});
    }
  });
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // the LDS ring is free (a partial tile's loop may follow)
}

// partial tiles of the LDS-DMA kernel (the last tile row / column of a
// launch, or Kd % BK != 0): predicated register loads, one LDS buffer per
// operand (A in ring0, B in ring1, rows padded to BK + 4), two barriers per
// k-chunk -- rare tiles, plain code
template <int BM, int BN, int WGM, int WGN, int BK, int NST, int TM, int TN>
__device__ __forceinline__ void sgemm_glds_fallback(const GemmArgsT<float>& g, int i0, int j0, float* ring0,
                                                    float* ring1, float16_t (&acc)[TM][TN]) {
  constexpr int NTH = 64 * WGM * WGN, WM = BM / WGM, WN = BN / WGN, PADK = BK + 4;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WGN, wc = wave % WGN;
  Loader32<BM, BN, NTH, BK> ld;
  const int aoff = (wr * WM + (lane & 31)) * PADK + 4 * (lane >> 5);
  const int boff = (wc * WN + (lane & 31)) * PADK + 4 * (lane >> 5);
  const int nch = (g.Kd + BK - 1) / BK;
  for (int t = 0; t < nch; ++t) {
    ld.template load<false>(g, i0, j0, t * BK);
    __syncthreads();
    ld.store(ring0, ring1);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < BK / 8; ++q) {
      float4 af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = *reinterpret_cast<const float4*>(&ring0[aoff + a * 32 * PADK + 8 * q]);
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b] = *reinterpret_cast<const float4*>(&ring1[boff + b * 32 * PADK + 8 * q]);
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
  }
}

// RDA: the fragment reads in asm (see sgemm_tile_loop_glds)
template <int BM, int BN, int WGM, int WGN, int BK, int NST, int WPE, int EPI = EPI_SUB, bool RDA = false>
__global__ __launch_bounds__(64 * WGM * WGN) __attribute__((amdgpu_waves_per_eu(WPE))) void sgemm_nt_glds_kernel(
    GemmArgsT<float> g) {
  constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 32, TN = WN / 32;
  constexpr int PADK = BK + 4;
  constexpr int STAGE = (BM + BN) * BK, ROWS = BM > BN ? BM : BN;
  static_assert(WM % 32 == 0 && WN % 32 == 0 && BK % 8 == 0, "32 x 32 blocks, k groups of 8");
  // one __shared__ object per ring buffer: hipcc then knows the DMA into one
  // buffer does not alias the ds_reads of another (with one array it drains
  // vmcnt(0) before every read); the register-staged fallback reuses them
  static_assert(NST >= 2 && NST <= 3, "LDS ring of 2 or 3 stages");
  constexpr int RB = STAGE > ROWS * PADK ? STAGE : ROWS * PADK;
  __shared__ __attribute__((aligned(16))) float ring0[RB];
  __shared__ __attribute__((aligned(16))) float ring1[RB];
  __shared__ __attribute__((aligned(16))) float ring2[NST > 2 ? RB : 4];
  int bid = blockIdx.x;
  {
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
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WGN, wc = wave % WGN;
  float16_t acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  if (i0 + BM <= g.M && j0 + BN <= g.N && g.Kd % BK == 0)
    sgemm_tile_loop_glds<BM, BN, WGM, WGN, BK, NST, RDA>(g, i0, j0, ring0, ring1, ring2, acc);
  else
    sgemm_glds_fallback<BM, BN, WGM, WGN, BK, NST>(g, i0, j0, ring0, ring1, acc);
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

template <int BM, int BN, int WGM, int WGN, int BK, int WPE, int EPI = EPI_SUB, int NST = 0, bool RDA = false>
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
  if constexpr (NST > 0)  // LDS-DMA staging, NST-deep ring (batch strides not supported)
    hipLaunchKernelGGL((sgemm_nt_glds_kernel<BM, BN, WGM, WGN, BK, NST, WPE, EPI, RDA>), dim3((unsigned)nblk), dim3(64 * WGM * WGN),
                       0, st, g);
  else
    hipLaunchKernelGGL((sgemm_nt_kernel<BM, BN, WGM, WGN, BK, WPE, EPI>), dim3((unsigned)nblk, (unsigned)batch),
                       dim3(64 * WGM * WGN), 0, st, g);
  return hipGetLastError();
}

}  // namespace ipmz
