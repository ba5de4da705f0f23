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
// the shortest chain per pivot.  The block is split into 4 block columns of
// 16; the chain is four COLUMN PASSES on wave 0 (colpass16: every remaining
// row of the block column eliminated element by element at once, row per
// lane, pivot column broadcast with v_readlane -- no TRSM step, no inverse
// on the chain) separated by the v_mfma_f64_16x16x4 update of the next block
// column's tiles (A: row l&15, k l>>4; C/D: col l&15, row (l>>4) + 4 reg):
//   pass p   : L[16p:, 16p:16p+16], D_p                          (wave 0)
//   A(p)     : A_i,p+1 -= L_ip (L_p+1,p D_p)^T, i > p            (3 - p waves)
//   B(p)     : pass p+1 on wave 0; the other tiles A_ij, p+2 <= j <= i, and
//              the inverse tiles X_pp (inv16), X_pj = -X_pp sum L_pk X_kj on
//              waves 1..3 in the pass's shadow
// X = L^{-1} is an output (the panel TRSM and the solve use it), not an
// input of the factor.  Stage clocks (kbench pieces): 36 k -> 32-36 k cycles
// for the block against the earlier leaf16 + TRSM-panel chain.  Arithmetic is
// the reference's order within a block column (LinearSolvers.cpp:26-36:
// zero-pivot rule, A[r][c] -= l_r w_c); across block columns the MFMA sums
// 16-term chunks first (1e-16-level rounding changes).
namespace diag64 {
constexpr int DS = 65;  // LDS row stride (doubles) of the 64 x 64 staging arrays

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
// One wave eliminates block column p (columns 16p .. 16p+15) of rows
// 16p .. 63 (lane l: row 16p + l): the reference's right-looking update
// A[r][j] -= l_r w_j with l_r = A[r][k] / d_k, w_j = A[j][k] (LinearSolvers.cpp:
// 22-36; zero-pivot rule), the pivot and the w_j read from the pivot
// column's lanes (v_readlane, wave-uniform), every row of the column updated
// together.  Writes L (strict lower part of the column) back to M and the
// pivots to dsh.  Upper entries of the diagonal tile are not meaningful.
__device__ __forceinline__ void colpass16(double* M, double* dsh, int p, int lane) {
  const int row = 16 * p + lane;
  const bool act = row < 64;
  const int rr = act ? row : 63;
  double v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = M[rr * DS + 16 * p + j];
  double dreg = 1.0;
  static_for<16>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const double draw = readlane_t(v[k], k);
    const double dk = draw == 0.0 ? 1e-8 : draw;  // LinearSolvers.cpp:26-28
    const double rdk = fast_rcp(dk);
    dreg = lane == k ? dk : dreg;
    const double l = lane > k ? v[k] * rdk : 0.0;
    static_for<15 - k>([&](auto jc) {
      constexpr int j = k + 1 + decltype(jc)::value;
      v[j] = fma(-l, readlane_t(v[k], j), v[j]);  // w_j = A[j][k], row j = lane j
    });
    v[k] = lane > k ? l : v[k];
  });
  if (act) {
#pragma unroll
    for (int j = 0; j < 16; ++j) M[rr * DS + 16 * p + j] = v[j];
  }
  if (lane < 16) dsh[16 * p + lane] = dreg;
}
// The pass every factor uses (CPV = 1): the pivot's reciprocal off the critical chain: every
// lane computes the (zero-rule) reciprocal of its own v[k+1] as soon as step
// k has updated it -- lane k+1's value is the next pivot -- so the v_rcp +
// Newton chain runs beside step k's remaining updates, and step k+1 starts
// from two readlanes.  The same operations on the same values: bitwise the
// same factor.
__device__ __forceinline__ void colpass16_spec(double* M, double* dsh, int p, int lane) {
  const int row = 16 * p + lane;
  const bool act = row < 64;
  const int rr = act ? row : 63;
  double v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = M[rr * DS + 16 * p + j];
  double dreg = 1.0, dl, rl;
  auto piv = [&](double x) {
    dl = x == 0.0 ? 1e-8 : x;  // LinearSolvers.cpp:26-28
    rl = fast_rcp(dl);
  };
  piv(v[0]);
  static_for<16>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const double dk = readlane_t(dl, k);
    const double rdk = readlane_t(rl, k);
    dreg = lane == k ? dk : dreg;
    const double l = lane > k ? v[k] * rdk : 0.0;
    if constexpr (k + 1 < 16) {
      v[k + 1] = fma(-l, readlane_t(v[k], k + 1), v[k + 1]);
      piv(v[k + 1]);
    }
    static_for<(k + 2 < 16 ? 14 - k : 0)>([&](auto jc) {
      constexpr int j = k + 2 + decltype(jc)::value;
      v[j] = fma(-l, readlane_t(v[k], j), v[j]);  // w_j = A[j][k], row j = lane j
    });
    v[k] = lane > k ? l : v[k];
  });
  if (act) {
#pragma unroll
    for (int j = 0; j < 16; ++j) M[rr * DS + 16 * p + j] = v[j];
  }
  if (lane < 16) dsh[16 * p + lane] = dreg;
}
// The same pass with a shorter dependent chain per pivot.  The pass time is
// the chain's latency (fewer instructions per step did not move it, round 6),
// and the chain was readlane(1/d_k) -> l = v_k / d_k -> v_{k+1} -= l w ->
// zero test -> select -> rcp -> two Newton steps.  Here the column-(k+1)
// update is v_{k+1} -= (v_k w) / d_k with v_k w formed off the chain (v_k
// and w are final one step earlier), and the zero rule is applied to the
// reciprocal (1 / 1e-8 selected after the rcp, the test beside it):
// readlane -> fma -> rcp -> NEWTON x (2 fma) -> select.  Other columns as in
// colpass16_spec.  Rounding differs from it at the 1e-16 level (the product
// order of the column-(k+1) update).
template <int NEWTON>
__device__ __forceinline__ void colpass16_short(double* M, double* dsh, int p, int lane) {
  const int row = 16 * p + lane;
  const bool act = row < 64;
  const int rr = act ? row : 63;
  double v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = M[rr * DS + 16 * p + j];
  const double rz = fast_rcp(1e-8);  // LinearSolvers.cpp:26-28: a zero pivot is 1e-8
  double dreg = 1.0, rl;
  auto piv = [&](double x) {
    double r = __builtin_amdgcn_rcp(x);
#pragma unroll
    for (int it = 0; it < NEWTON; ++it) r = fma(r, fma(-x, r, 1.0), r);
    rl = x == 0.0 ? rz : r;
  };
  piv(v[0]);
  static_for<16>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const double rdk = readlane_t(rl, k);
    dreg = lane == k ? (v[k] == 0.0 ? 1e-8 : v[k]) : dreg;
    if constexpr (k + 1 < 16) {
      const double t = v[k] * readlane_t(v[k], k + 1);
      v[k + 1] = fma(-t, rdk, v[k + 1]);
      piv(v[k + 1]);
    }
    const double l = lane > k ? v[k] * rdk : 0.0;
    static_for<(k + 2 < 16 ? 14 - k : 0)>([&](auto jc) {
      constexpr int j = k + 2 + decltype(jc)::value;
      v[j] = fma(-l, readlane_t(v[k], j), v[j]);  // w_j = A[j][k], row j = lane j
    });
    v[k] = lane > k ? l : v[k];
  });
  if (act) {
#pragma unroll
    for (int j = 0; j < 16; ++j) M[rr * DS + 16 * p + j] = v[j];
  }
  if (lane < 16) dsh[16 * p + lane] = dreg;
}
// X_pp = L_pp^{-1} of a unit-lower 16 x 16 tile: lane c (mod 16) solves
// L x = e_c right-looking (L entries are wave-uniform LDS broadcasts)
__device__ __forceinline__ void inv16(const double* Lt, double* Xt, int lane) {
  const int c = lane & 15;
  double x[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) x[r] = r == c ? 1.0 : 0.0;
  static_for<15>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    static_for<15 - j>([&](auto rc) {
      constexpr int r = j + 1 + decltype(rc)::value;
      x[r] = fma(-Lt[r * DS + j], x[j], x[r]);
    });
  });
  if (lane < 16) {
#pragma unroll
    for (int r = 0; r < 16; ++r) Xt[r * DS + c] = x[r];
  }
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
// PRE_WB: called by every thread once L, D and X are final in LDS, before
// their write-back (the panel chain issues the next block's operand loads
// there, so their latency overlaps the write-back's stores).
struct NoHook {
  __device__ void operator()() const {}
};
// Ksrc (optional): read the block from there instead of K (the batched
// factor's first touch of the assembled KKT, small.hip); L is written to K.
// tid_arg (optional): the caller's thread index (small.hip launders it per
// block column so the body's lane-dependent addresses are not hoisted).
// WB_LINV = false: L^{-1} is not written back (the caller writes it from X
// later, small.hip); IDLE0: called by waves 1.. while wave 0 runs the first
// column pass (the batched factor writes the previous block's L^{-1} there).
// abort8: see the loop below.  POST2: called by every thread after the
// barrier that follows the first column pass (with DRAIN0: every earlier
// store of the workgroup is complete there -- the 4-wave panel chain raises
// the previous block's flags in it).  DRAIN0: every wave drains its outstanding global stores (vmcnt(0)) before
// the barrier after the first column pass -- wave 0 after its pass, so the
// wait is off its chain.  WB_D = false: D (and the non-finite pivot check)
// is left to the caller too (the 8-wave panel chain writes D and L^{-1} from
// its other wave group, off the critical path).
template <bool COH, bool LSC = false, typename TS = double, bool PRE = false, int NW = 4, typename PRE_WB = NoHook,
          bool WB_LINV = true, typename IDLE0 = NoHook, int CPV = 1, bool DRAIN0 = false, bool WB_D = true,
          typename POST2 = NoHook>
__device__ __forceinline__ void diag64_body(TS* __restrict__ K, int64_t ld, int k0, int b, TS* __restrict__ D,
                                            TS* __restrict__ Linv, int* __restrict__ info, double* M, double* X,
                                            double* dsh, unsigned long long* clkbuf, PRE_WB pre_wb = PRE_WB(),
                                            const TS* __restrict__ Ksrc = nullptr, int tid_arg = -1,
                                            IDLE0 idle0 = IDLE0(), const volatile unsigned* abort8 = nullptr,
                                            POST2 post2 = POST2()) {
  // wave: readfirstlane makes the wave roles below uniform branches for the
  // compiler (threadIdx.x-derived values are divergent to it), so the roles'
  // register live ranges do not overlap
  const int tid = tid_arg < 0 ? (int)threadIdx.x : tid_arg, lane = tid & 63,
            wave = __builtin_amdgcn_readfirstlane(tid >> 6);
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
      const TS* src = &(Ksrc ? Ksrc : K)[(int64_t)(k0 + r2) * ld + k0 + c2];
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
  // Critical chain: four COLUMN PASSES (wave 0), each eliminating a 16-column
  // block column of every remaining row at once (so no TRSM step and no
  // inverse on the chain), separated by the MFMA update of the next block
  // column.  The inverse X = L^{-1} (a consumer output, not an input of the
  // factor) and the non-critical tile updates run on the other waves in the
  // shadow of the passes.
  auto upd = [&](int i, int j, int p) {  // A_ij -= L_ip (L_jp D_p)^T
    double4_t acc = tile_load(Mt(i, j), lane);
    acc = tile_nt_lds(Mt(i, p), Mt(j, p), &dsh[16 * p], acc, lane);
    tile_store(Mt(i, j), acc, lane);
  };
  auto xsum = [&](int p, int j) {  // S = sum_{k=j}^{p-1} L_pk X_kj
    double4_t sacc = {0.0, 0.0, 0.0, 0.0};
    for (int k = j; k < p; ++k) sacc = tile_nn(Mt(p, k), Xt(k, j), sacc, lane);
    return sacc;
  };
  auto xmul = [&](int p, int j, double4_t sacc) {  // X_pj = -X_pp S
    // S in accumulator layout IS the NN B-fragment
    double4_t acc = {0.0, 0.0, 0.0, 0.0};
    const double* xp = Xt(p, p);
#pragma unroll
    for (int q = 0; q < 4; ++q) acc = mfma_f64_16x16x4(-xp[(lane & 15) * DS + 4 * q + (lane >> 4)], sacc[q], acc);
    tile_store(Xt(p, j), acc, lane);
  };
  auto xoff = [&](int p, int j) { xmul(p, j, xsum(p, j)); };  // X_pj = -X_pp sum_{k=j}^{p-1} L_pk X_kj
  auto colpass = [&](int p) {
    if constexpr (CPV == 1) colpass16_spec(M, dsh, p, lane);
    else if constexpr (CPV == 3) colpass16_short<2>(M, dsh, p, lane);
    else if constexpr (CPV == 4) colpass16_short<1>(M, dsh, p, lane);
    else colpass16(M, dsh, p, lane);
  };
  if (wave == 0) colpass(0);
  else idle0();
  if constexpr (DRAIN0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  post2();  // (every thread, after the barrier that follows the first column pass)
  clk();
  for (int p = 0; p < 3; ++p) {
    // ---- A(p): the critical tiles (i, p+1), i > p, with block column p
    if (wave < 3 - p) upd(p + 1 + wave, p + 1, p);
    __syncthreads();
    clk();
    // ---- B(p): pass p+1 on wave 0; the other tiles (i, j), p+2 <= j <= i,
    // with block column p, and the inverse tiles of block row p (X_pp, then
    // X_pj, j < p, on one wave: they depend on X_pp) -- all in the pass's shadow
    if (wave == 0) {
      colpass(p + 1);
    } else if (wave < 4) {
      if (p == 0) {  // tiles (2,2), (3,2), (3,3) on waves 1..3; X_00 after wave 1's tile
        const int i = wave == 1 ? 2 : 3, j = wave == 3 ? 3 : 2;
        upd(i, j, 0);
        if (wave == 1) inv16(Mt(0, 0), Xt(0, 0), lane);
      } else if (p == 1) {  // tile (3,3); X_11, X_10
        if (wave == 1) upd(3, 3, 1);
        if (wave == 2) {
          inv16(Mt(1, 1), Xt(1, 1), lane);
          xoff(1, 0);
        }
      } else if (wave == 1) {  // X_22, X_20, X_21
        inv16(Mt(2, 2), Xt(2, 2), lane);
        xoff(2, 0);
        xoff(2, 1);
      }
    }
    __syncthreads();
    clk();
    // abort8 (LDS, set before the 8th barrier): the caller gives the block up
    // (the 8-wave panel chain's launch found itself alone, panel.hip)
    if (p == 2 && abort8 && *abort8) return;
  }
  // ---- the last row of inverse tiles: X_33 on wave 0 while waves 1..3 sum
  // S_3j = sum_k L_3k X_kj (X_33 is not needed for those), then X_3j = -X_33 S_3j
  double4_t s3 = {0.0, 0.0, 0.0, 0.0};
  if (wave == 0) inv16(Mt(3, 3), Xt(3, 3), lane);
  else if (wave < 4) s3 = xsum(3, wave - 1);
  __syncthreads();
  if (wave >= 1 && wave < 4) xmul(3, wave - 1, s3);
  __syncthreads();
  clk();
  pre_wb();
  // write back L (strict lower), D, and L^{-1} (64 x 64 row-major, identity-padded)
#pragma unroll 4
  for (int idx = tid; idx < 64 * 64; idx += 64 * NW) {
    const int rr = idx >> 6, cc = idx & 63;
    if (rr < b && cc < rr) K[(int64_t)(k0 + rr) * ld + k0 + cc] = (TS)M[rr * DS + cc];
    if constexpr (WB_LINV) {
      const TS x = (TS)(cc > rr ? 0.0 : ((rr >= b || cc >= b) ? (rr == cc ? 1.0 : 0.0) : X[rr * DS + cc]));
      if constexpr (COH) __hip_atomic_store(&Linv[idx], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else Linv[idx] = x;
    }
  }
  if (WB_D && tid < b) {
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
