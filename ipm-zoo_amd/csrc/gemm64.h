// fp64 NT GEMM with LDS-DMA operand staging: the trailing update
// A22 -= W21 L21^T of the fp64 LDL^T (LinearSolvers.cpp:30-36, rank nbo) for
// launches whose tiles are all full (M, N multiples of the tile, Kd of BK) --
// the rest keep the register-staged engine of gemm.h.
//
// Against gemm.h's kernel (register staging, one float2 / double2 per thread
// per chunk, a ds_write pass, one barrier per 16-deep chunk, ds_read_b64
// fragments):
//   * the operands go global -> LDS by global_load_lds_dwordx4 (no staging
//     VGPRs, no ds_write), through an NST-deep ring whose later stages stay in
//     flight across the barrier (counted vmcnt, raw s_barrier);
//   * the fragments are read with ds_read_b128: lane l holds k = 2 (l >> 4)
//     + {0, 1} of an 8-deep k group for TWO v_mfma_f64_16x16x4 (MFMA s takes
//     element s on both operands), half the LDS read instructions;
//   * the LDS image is unpadded [rows][BK doubles] with the 16-byte slots of
//     a row XOR-swizzled by a function of the row (the DMA writes 1 KB
//     lane-linearly, so the swizzle sits on each lane's SOURCE address);
//     every ds_read_b128 lane group hits 16 distinct bank slots
//     (brute-force checked for BK = 8 and 16, the two depths used);
//   * the fragment reads are inline asm, so hipcc's wait insertion (which
//     drains every DMA in flight before a compiler-visible LDS read) stays
//     out of the k loop; the reads are waited for by hand.
// The k order of the sums differs from gemm.h's (pairs of MFMAs per 8-deep
// group), the result is deterministic run to run.
#pragma once
#include "common.h"
#include "gemm.h"
#include "gemm32.h"  // vmcnt_lgkm0, lds_addr helpers

namespace ipmz {

typedef double f64x2 __attribute__((ext_vector_type(2)));

// XOR applied to the 16-byte slot index of row r (BK doubles per row)
template <int BK>
__device__ __forceinline__ int glds_swz64(int r) {
  if constexpr (BK == 8) return (0x1320 >> (4 * ((r >> 2) & 3))) & 3;  // {0, 2, 3, 1}[(r >> 2) & 3]
  else return (r >> 1) & 7;                                              // BK = 16
}
__device__ __forceinline__ unsigned lds_addr64(const double* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) double*)p;
}

template <int BM, int BN, int WGM, int WGN, int BK, int NST, int WPE, int EPI = EPI_SUB>
__global__ __launch_bounds__(64 * WGM * WGN) __attribute__((amdgpu_waves_per_eu(WPE))) void dgemm_nt_glds_kernel(
    GemmArgsT<double> g) {
  constexpr int NW = WGM * WGN, WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  constexpr int SLOTS = BK / 2, RPI = 64 / SLOTS;  // 16-byte slots per row, rows per DMA wave-instruction
  constexpr int IA = BM / RPI, IB = BN / RPI;       // DMA instructions per stage
  constexpr int LPW = (IA + IB) / NW;               // per wave per stage
  constexpr int STAGE = (BM + BN) * BK;             // doubles per stage
  static_assert(BK == 8 || BK == 16, "swizzles checked for BK 8 and 16");
  static_assert((IA + IB) % NW == 0 && WM % 16 == 0 && WN % 16 == 0, "tile shape");
  static_assert(NST >= 2 && NST <= 3, "LDS ring of 2 or 3 stages");
  // one __shared__ object per ring buffer
  __shared__ __attribute__((aligned(16))) double ring0[STAGE];
  __shared__ __attribute__((aligned(16))) double ring1[STAGE];
  __shared__ __attribute__((aligned(16))) double ring2[NST > 2 ? STAGE : 2];
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
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave / WGN, wc = wave % WGN;
  const int nch = g.Kd / BK;
  const int rl = lane / SLOTS, phys = lane % SLOTS;

  double4_t acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = (double4_t){0.0, 0.0, 0.0, 0.0};

  auto ring = [&](auto bc) -> double* {
    constexpr int B = decltype(bc)::value;
    if constexpr (B == 0) return ring0;
    else if constexpr (B == 1) return ring1;
    else return ring2;
  };
  auto issue = [&](int t, auto bc) {
    double* st = ring(bc);
    const int kk = t * BK;
#pragma unroll
    for (int u = 0; u < LPW; ++u) {
      const int m = wave + NW * u;
      const double* src;
      double* dst;
      if (m < IA) {
        const int r = m * RPI + rl;
        src = g.A + (int64_t)(i0 + r) * g.lda + kk + 2 * (phys ^ glds_swz64<BK>(r));
        dst = st + m * 128;
      } else {
        const int r = (m - IA) * RPI + rl;
        src = g.B + (int64_t)(j0 + r) * g.ldb + kk + 2 * (phys ^ glds_swz64<BK>(r));
        dst = st + BM * BK + (m - IA) * 128;
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };
  auto rd_asm = [&](const double* as, const double* bs, int q, f64x2 (&af)[TM], f64x2 (&bf)[TN]) {
    const int c = 4 * q + (lane >> 4);
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int r = wr * WM + a * 16 + (lane & 15);
      asm volatile("ds_read_b128 %0, %1"
                   : "=v"(af[a])
                   : "v"(lds_addr64(&as[r * BK + 2 * (c ^ glds_swz64<BK>(r))]))
                   : "memory");
    }
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int r = wc * WN + b * 16 + (lane & 15);
      asm volatile("ds_read_b128 %0, %1"
                   : "=v"(bf[b])
                   : "v"(lds_addr64(&bs[r * BK + 2 * (c ^ glds_swz64<BK>(r))]))
                   : "memory");
    }
  };
  // wait for the asm reads in flight; the MFMAs issued so far stay before the
  // wait (their accumulators tied to it), the fragments' uses after it
  auto wait_rd = [&](f64x2 (&af)[TM], f64x2 (&bf)[TN]) {
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
  auto mm = [&](const f64x2 (&af)[TM], const f64x2 (&bf)[TN]) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = mfma_f64_16x16x4(af[a][s], bf[b][s], acc[a][b]);
  };
  // group q + 1's fragment reads in flight during group q's MFMAs
  auto compute = [&](auto bc) {
    const double* as = ring(bc);
    const double* bs = as + BM * BK;
    f64x2 af0[TM], bf0[TN], af1[TM], bf1[TN];
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
  };
  static_for<NST - 1>([&](auto sc) {
    if (decltype(sc)::value < nch) issue(decltype(sc)::value, sc);
  });
  int t0 = 0;
  for (; t0 + 2 * (NST - 1) < nch; t0 += NST) {  // steady state: every stage issued here exists
    static_for<NST>([&](auto sc) {
      constexpr int S = decltype(sc)::value;
      __builtin_amdgcn_s_waitcnt(vmcnt_lgkm0((NST - 2) * LPW));  // stage t0 + S landed, later ones in flight
      __builtin_amdgcn_s_barrier();
      issue(t0 + S + NST - 1, std::integral_constant<int, (S + NST - 1) % NST>{});  // stage t - 1's buffer
      compute(sc);
    });
  }
  static_for<2 * NST - 1>([&](auto uc) {  // tail: waits counted down
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

  // epilogue: C -= acc (f64 C/D layout: column lane & 15, row (lane >> 4) + 4 reg)
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int j = j0 + wc * WN + b * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + wr * WM + a * 16 + Mfma<double>::row(lane, r);
        double* cp = g.C + (int64_t)i * g.ldc + j;
        *cp = *cp - acc[a][b][r];
      }
    }
}

// full tiles only; false: not launched (the caller takes gemm.h's kernel)
// lds_pad: extra (dynamic, unused) LDS bytes per workgroup -- caps the
// workgroups per CU by LDS (experiment: room for a panel workgroup beside one)
template <int BM, int BN, int WGM, int WGN, int BK, int NST, int WPE, int EPI = EPI_SUB>
static bool launch_dgemm_glds(GemmArgsT<double> g, hipStream_t st, hipError_t& e, unsigned lds_pad = 0) {
  if (g.M % BM || g.N % BN || g.Kd % BK || g.Kd == 0 || g.M == 0 || g.N == 0) return false;
  if (((reinterpret_cast<uintptr_t>(g.A) | reinterpret_cast<uintptr_t>(g.B)) & 15) || (g.lda | g.ldb) & 1) return false;
  g.ntm = g.M / BM;
  g.ntn = g.N / BN;
  int64_t nblk = (int64_t)g.ntm * g.ntn;
  if (g.lower == 2) {
    if (BM == BN) nblk = (int64_t)g.ntm * (g.ntm + 1) / 2;
    else g.lower = 1;
  }
  hipLaunchKernelGGL((dgemm_nt_glds_kernel<BM, BN, WGM, WGN, BK, NST, WPE, EPI>), dim3((unsigned)nblk),
                     dim3(64 * WGM * WGN), lds_pad, st, g);
  e = hipGetLastError();
  return true;
}

}  // namespace ipmz
