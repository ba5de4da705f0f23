// Diagonal-block LDL^T (64 x 64) on fp64 MFMA: shared by the stand-alone
// diag kernel (ldlt.hip) and the fused panel-step kernel (panel.hip).
#pragma once
#include "common.h"
#include "sync.h"

namespace ipmz {

// ---------------------------------------------------------------------------
// Diagonal block, NB = 64, blocked on fp64 MFMA (the default for nbi = 64).
//
// The 64 pivots are sequential whatever the kernel does, so the design goal is
// the shortest chain per pivot: the block is split into 4 x 4 tiles of 16 and
// only the 16-pivot leaves run element by element, inside ONE wave with no
// memory traffic at all (row-per-lane, DPP row_share broadcasts, readlane of
// the pivot).  Everything between leaves is 16 x 16 x 16 tile products on
// v_mfma_f64_16x16x4 spread over the 4 waves (A/B fragment: row l&15,
// k l>>4; C/D: col l&15, row (l>>4) + 4 reg), with one workgroup barrier per
// stage (8 in all):
//   leaf  p : L_pp, D_p, X_pp = L_pp^{-1}                       (wave 0)
//   panel p : T = A_ip X_pp^T, L_ip = T / D_p              (i > p)
//             X_pj = -X_pp sum_{k=j}^{p-1} L_pk X_kj       (j < p)
//   update p: A_ij -= L_ip (L_jp D_p)^T (p < j <= i); wave 0 takes (p+1, p+1) first
//             and goes straight on to leaf p+1
// X = L^{-1} (the block inverse the panel TRSM and the solve use) falls out of
// the same tiles.  Leaf arithmetic is the reference's order
// (LinearSolvers.cpp:26-36: zero-pivot rule, A[r][c] -= l_r w_c); across
// tiles the MFMA sums 16-term chunks first (1e-16-level rounding changes).
namespace diag64 {
constexpr int DS = 65;  // LDS row stride (doubles) of the 64 x 64 staging arrays

// Wave-level 16 x 16 LDL^T + inverse of the tile at T (row stride DS).  All
// four 16-lane row groups compute the same thing (lane l: row l & 15); row
// group 0 stores L (strict lower) back into T, D into dout, X = L^{-1} into Xt.
__device__ __forceinline__ void leaf16(double* T, double* Xt, double* dout, int lane) {
  const int r = lane & 15;
  double v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = T[r * DS + j];
  double dreg = 1.0;
  static_for<16>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const double draw = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v[k]), k),
                                         __builtin_amdgcn_readlane(__double2loint(v[k]), k));
    const double dk = draw == 0.0 ? 1e-8 : draw;  // LinearSolvers.cpp:26-28
    const double rdk = fast_rcp(dk);
    dreg = r == k ? dk : dreg;
    const double l = v[k] * rdk;
    static_for<15 - k>([&](auto jc) {
      constexpr int j = k + 1 + decltype(jc)::value;
      v[j] = fma(-l, dpp_bcast<0x150 + j>(v[k]), v[j]);  // row_share:j -> w_j
    });
    v[k] = l;
  });
  // X = L^{-1}, row r: x_r -= L[r][j] x_j for j < r (right-looking over j)
  double x[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) x[c] = c == r ? 1.0 : 0.0;
  static_for<15>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const double m = r > j ? v[j] : 0.0;
    static_for<j + 1>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      x[c] = fma(-m, dpp_bcast<0x150 + j>(x[c]), x[c]);
    });
  });
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j < r) T[r * DS + j] = v[j];
      Xt[r * DS + j] = x[j];
    }
    dout[r] = dreg;
  }
}

// acc += P Q^T over 16 (NT: both operands row-major 16 x 16 tiles, stride DS)
__device__ __forceinline__ double4_t tile_nt(const double* P, const double* Q, double4_t acc, int lane, bool negP) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = 4 * q + (lane >> 4);
    const double a = P[(lane & 15) * DS + k];
    acc = mfma_f64_16x16x4(negP ? -a : a, Q[(lane & 15) * DS + k], acc);
  }
  return acc;
}
// acc -= P (Q diag(dq))^T over 16: the W = L D operand formed on the fly
// from the L tile and the pivots (no separate W tile in LDS)
__device__ __forceinline__ double4_t tile_nt_lds(const double* P, const double* Q, const double* dq, double4_t acc,
                                                 int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = 4 * q + (lane >> 4);
    acc = mfma_f64_16x16x4(-P[(lane & 15) * DS + k], Q[(lane & 15) * DS + k] * dq[k], acc);
  }
  return acc;
}
// acc += P Q over 16 (NN)
__device__ __forceinline__ double4_t tile_nn(const double* P, const double* Q, double4_t acc, int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = 4 * q + (lane >> 4);
    acc = mfma_f64_16x16x4(P[(lane & 15) * DS + k], Q[k * DS + (lane & 15)], acc);
  }
  return acc;
}
__device__ __forceinline__ double4_t tile_load(const double* C, int lane) {
  double4_t v;
#pragma unroll
  for (int g = 0; g < 4; ++g) v[g] = C[((lane >> 4) + 4 * g) * DS + (lane & 15)];
  return v;
}
__device__ __forceinline__ void tile_store(double* C, double4_t v, int lane) {
#pragma unroll
  for (int g = 0; g < 4; ++g) C[((lane >> 4) + 4 * g) * DS + (lane & 15)] = v[g];
}
}  // namespace diag64
using namespace diag64;

// The whole diagonal-block factorization for one 256-thread workgroup.
// LDS: M, X (64 x DS each) and dsh (64) -- 66.5 KB, so a workgroup running
// this fits the LDS slot one trailing-GEMM tile frees (73.7 KB) and a
// high-priority panel launch is not starved behind a whole GEMM launch.
// LSC: read the block with agent-scope loads (it was written earlier in the
// same launch, possibly through another CU's L1).  COH: Linv and D are stored
// write-through (agent-scope relaxed atomics) for consumers in other
// workgroups of the same launch.  clk != nullptr records stage clocks.
// TS: storage type of K, D and L^{-1} (float for the fp32 factor of the
// mixed-precision path: the 64 x 64 block itself is factored in fp64).
// PRE: the block is already in M (row stride DS, lower triangle, upper
// zero, identity padding past b) -- handed over through LDS by its producer.
// NW: waves in the workgroup (4 or 8); waves >= 4 only load/store and join
// the barriers.
template <bool COH, bool LSC = false, typename TS = double, bool PRE = false, int NW = 4>
__device__ __forceinline__ void diag64_body(TS* __restrict__ K, int64_t ld, int k0, int b, TS* __restrict__ D,
                                            TS* __restrict__ Linv, int* __restrict__ info, double* M, double* X,
                                            double* dsh, unsigned long long* clkbuf) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  auto Mt = [&](int i, int j) { return &M[(16 * i) * DS + 16 * j]; };
  auto Xt = [&](int i, int j) { return &X[(16 * i) * DS + 16 * j]; };
  int nclk = 0;
  auto clk = [&]() {
    if (clkbuf && tid == 0) clkbuf[nclk] = __builtin_amdgcn_s_memtime();
    ++nclk;
  };
  clk();
  // coalesced load, identity padding past b; X upper tiles are never read
  if constexpr (!PRE) {
    constexpr int NQ = 64 / NW;
    double t[NQ];  // all loads in flight: addresses clamped into the valid triangle
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int rr = (tid >> 6) + NW * q, cc = tid & 63;
      const int r2 = rr < b ? rr : 0, c2 = cc <= r2 ? cc : 0;
      const TS* src = &K[(int64_t)(k0 + r2) * ld + k0 + c2];
      t[q] = (double)(LSC ? ld_sc1(src) : *src);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int rr = (tid >> 6) + NW * q, cc = tid & 63;
      M[rr * DS + cc] = (rr < b && cc <= rr) ? t[q] : (rr == cc ? 1.0 : 0.0);
    }
  }
  __syncthreads();
  clk();
  if (wave == 0) leaf16(Mt(0, 0), Xt(0, 0), &dsh[0], lane);
  __syncthreads();
  clk();
  for (int p = 0; p < 4; ++p) {
    // ---- panel p: TRSM tiles i > p and inverse tiles X_pj, j < p (3 in all)
    {
      const int t = wave;  // tiles 0..2
      if (t < 3) {
        if (t < 3 - p) {
          const int i = p + 1 + t;
          double4_t acc = tile_nt(Mt(i, p), Xt(p, p), (double4_t){0.0, 0.0, 0.0, 0.0}, lane, false);
          const double rc = 1.0 / dsh[16 * p + (lane & 15)];
#pragma unroll
          for (int g = 0; g < 4; ++g) acc[g] = acc[g] * rc;
          tile_store(Mt(i, p), acc, lane);
        } else {
          const int j = t - (3 - p);  // 0 .. p-1
          double4_t s = {0.0, 0.0, 0.0, 0.0};
          for (int k = j; k < p; ++k) s = tile_nn(Mt(p, k), Xt(k, j), s, lane);
          // X_pj = -X_pp S: S in accumulator layout IS the NN B-fragment
          double4_t acc = {0.0, 0.0, 0.0, 0.0};
          const double* xp = Xt(p, p);
#pragma unroll
          for (int q = 0; q < 4; ++q) acc = mfma_f64_16x16x4(-xp[(lane & 15) * DS + 4 * q + (lane >> 4)], s[q], acc);
          tile_store(Xt(p, j), acc, lane);
        }
      }
    }
    __syncthreads();
    clk();
    if (p == 3) break;
    // ---- update p: A_ij -= L_ip W_jp^T, p < j <= i; wave 0: (p+1, p+1) then leaf p+1
    if (wave == 0) {
      const int d = p + 1;
      double4_t acc = tile_load(Mt(d, d), lane);
      acc = tile_nt_lds(Mt(d, p), Mt(d, p), &dsh[16 * p], acc, lane);
      tile_store(Mt(d, d), acc, lane);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      clk();
      leaf16(Mt(d, d), Xt(d, d), &dsh[16 * d], lane);
    } else {
      int t = 0;
      for (int i = p + 1; i < 4; ++i)
        for (int j = p + 1; j <= i; ++j) {
          if (i == p + 1 && j == p + 1) continue;
          if (t++ % 3 != wave - 1) continue;
          double4_t acc = tile_load(Mt(i, j), lane);
          acc = tile_nt_lds(Mt(i, p), Mt(j, p), &dsh[16 * p], acc, lane);
          tile_store(Mt(i, j), acc, lane);
        }
    }
    __syncthreads();
    clk();
  }
  // write back L (strict lower), D, and L^{-1} (64 x 64 row-major, identity-padded)
#pragma unroll 4
  for (int idx = tid; idx < 64 * 64; idx += 64 * NW) {
    const int rr = idx >> 6, cc = idx & 63;
    if (rr < b && cc < rr) K[(int64_t)(k0 + rr) * ld + k0 + cc] = (TS)M[rr * DS + cc];
    const TS x = (TS)(cc > rr ? 0.0 : ((rr >= b || cc >= b) ? (rr == cc ? 1.0 : 0.0) : X[rr * DS + cc]));
    if constexpr (COH) __hip_atomic_store(&Linv[idx], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else Linv[idx] = x;
  }
  if (tid < b) {
    const double dk = dsh[tid];
    if constexpr (COH) __hip_atomic_store(&D[k0 + tid], (TS)dk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else D[k0 + tid] = (TS)dk;
    if (!(fabs(dk) <= 1.7976931348623157e308)) atomicMin(info, k0 + tid + 1);  // first non-finite pivot
  }
  if (clkbuf) {
    __syncthreads();
    clk();
    if (tid == 0) clkbuf[31] = nclk;
  }
}


}  // namespace ipmz
