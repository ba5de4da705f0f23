// The panel path of the blocked LDL^T: for one outer panel (columns
// [k0, c1), nb <= 8 inner blocks of 64), the column loop of
// LinearSolvers::ldlt_decomposition (LinearSolvers.cpp:20-40) restricted to
// those columns, as roles that hand off by flags.  ONE kernel (panel_kernel,
// 66.5 KB of LDS) is launched twice -- on the chain stream and on the rows
// stream, after the look-ahead strip update of the rows below -- and every
// workgroup takes its role from ticket counters (the chain roles' shared by
// both launches; see panel_kernel for why that cannot deadlock):
//
//   chain roles (the panel's diagonal region, first updated with the previous
//   panel; s_setprio 3):
//     ticket 0 = the CHAIN: for every inner block j, factor the 64 x 64
//       diagonal block (diag64_body), publish DIAG[j], then -- still in its
//       own LDS, no hand-off -- the TRSM of the next region block (j+1, j)
//       and that block's own diagonal update; the result IS the next diagonal
//       block.  The whole critical path of the panel lives on one CU.
//     tickets nb.. = TILE WORKERS: one region block (c, q), c >= 1, each,
//       updated with the previous panel (flag TILE[c][q]); the chain updates
//       block (0, 0) itself, straight into its LDS image.
//     ticket c < nb = region HELPER c (rows of block c): the TRSMs of its
//       blocks j <= c - 2 and their strip updates, then READY[c]: its blocks
//       (c, c-1) and (c, c) carry every contribution but block c-1's, which
//       the chain applies itself.
//   rows roles (one per 64 rows below the region): for every j: TRSM with
//     L_jj^{-1} (waits DIAG[j]), L = T / D, W = T, and the strip pieces
//     A[rows, q] -= L W[q, j]^T (waits REG[j][q]).
//
// Flags: one area of IPMZ_PANEL_CTRL_WORDS words per outer panel (zeroed by
// one memset when the factorization starts); the sticky error word is shared.
// Hand-off protocol (cdna_hip_programming.md §6 Guideline 16, "Valid forms"
// row 1): data for another workgroup of a running launch is stored with sc1
// (relaxed agent-scope atomic stores), every storing wave drains vmcnt(0),
// a workgroup barrier, then one lane stores the flag; consumers poll with
// agent-scope loads and read the data with sc1 loads.
#include "common.h"
#include "diag64.h"
#include "kernels.h"
#include "sync.h"

namespace ipmz {

// -DIPMZ_CHAIN_STAMPS (tools/kbench "chainclk" only): s_memrealtime stamps of
// the chain role per 64-column block (k0 / 64 + j): 0 diag start, 1 READY[c]
// seen, 2 diag done (write-back included), 3 operands loaded, 4 TRSM done,
// 5 own update done (REG published); helpers: READY[c] published; rows role
// 0: start, end; launches: first workgroup start per launch.
__device__ unsigned long long g_cstamp[IPMZ_CHAIN_STAMP_BLOCKS][8];
__device__ unsigned long long g_hstamp[IPMZ_CHAIN_STAMP_BLOCKS][4];
#ifdef IPMZ_CHAIN_STAMPS
#define CSTAMP(jb, i) \
  if (threadIdx.x == 0 && (jb) < IPMZ_CHAIN_STAMP_BLOCKS) g_cstamp[jb][i] = __builtin_amdgcn_s_memrealtime()
#define HSTAMP(jb, i) \
  if (threadIdx.x == 0 && (jb) < IPMZ_CHAIN_STAMP_BLOCKS) g_hstamp[jb][i] = __builtin_amdgcn_s_memrealtime()
#else
#define CSTAMP(jb, i)
#define HSTAMP(jb, i)
#endif
hipError_t chain_stamps(unsigned long long* c, unsigned long long* h) {  // DEBUG
  hipError_t e = hipMemcpyFromSymbol(c, HIP_SYMBOL(g_cstamp), sizeof(g_cstamp));
  if (e != hipSuccess) return e;
  return hipMemcpyFromSymbol(h, HIP_SYMBOL(g_hstamp), sizeof(g_hstamp));
}

namespace {
enum { OP_TICKET = 0, OP_DIAG = 4, OP_REG = 16, OP_READY = 96, OP_TILE = 128 };
constexpr int OP_NBMAX = IPMZ_NBO_MAX / 64;
static_assert(OP_DIAG + OP_NBMAX <= OP_REG && OP_REG + OP_NBMAX * OP_NBMAX <= OP_READY, "ctrl layout");
static_assert(OP_READY + OP_NBMAX <= OP_TILE, "ctrl layout");
static_assert(OP_TILE + OP_NBMAX * OP_NBMAX <= IPMZ_PANEL_CTRL_WORDS, "panel ctrl area too small");

// A 64 x 64 tile in MFMA accumulator layout: wave w holds rows 16w + row(lane, g),
// columns 16n + (lane & 15), n, g in 0..3.
template <typename T>
using Acc4 = typename Mfma<T>::acc_t[4];

// acc[n] (+)= sgn * A[16w.., :] B[16n.., :]^T over k in [0, 64): A, B row-major
// 64 x DS tiles in LDS (B read through bf: a functor (row, k) -> T).
template <typename T, bool NEG, typename BF>
__device__ __forceinline__ void mma_tile(const T* As, BF bf, typename Mfma<T>::acc_t (&acc)[4]) {
  typedef Mfma<T> MF;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int arow = 16 * wave + (lane & 15);
#pragma unroll 4
  for (int s = 0; s < 16; ++s) {
    const int k = 4 * s + (lane >> 4);
    const T a = NEG ? -As[arow * DS + k] : As[arow * DS + k];
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[n] = MF::mma(a, bf(16 * n + (lane & 15), k), acc[n]);
  }
}

// acc[n] += A[16w.., :] B[16n.., :]^T for a LOWER-triangular B (the diagonal
// block's inverse): k-chunks past column block n's diagonal are zero and
// skipped (40 of 64 MFMAs per wave), the diagonal chunk masked through bf.
// The chain's TRSM step: 4.5 -> 2.5 us per block (kbench chain clocks).
template <typename T, typename BF>
__device__ __forceinline__ void mma_tile_lower(const T* As, BF bf, typename Mfma<T>::acc_t (&acc)[4]) {
  typedef Mfma<T> MF;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int arow = 16 * wave + (lane & 15);
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int k = 4 * s + (lane >> 4);
    const T a = As[arow * DS + k];
#pragma unroll
    for (int n = 0; n < 4; ++n)
      if (s < 4 * (n + 1)) acc[n] = MF::mma(a, bf(16 * n + (lane & 15), k), acc[n]);
  }
}

// 64 x 64 tile of a row-major matrix (ld) into LDS (rows < rows, columns <
// cols; zeros elsewhere): 16 loads in flight per thread.  SC: agent-scope
// loads (data written earlier in this launch, possibly by another CU).
template <typename T, bool SC>
__device__ __forceinline__ void stage_tile(T* dst, const T* src, int64_t ld, int rows, int cols) {
  const int tid = threadIdx.x;
  T v[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int rr = (tid >> 6) + 4 * q, cc = tid & 63;
    const T* p = &src[(int64_t)(rr < rows ? rr : 0) * ld + (cc < cols ? cc : 0)];
    v[q] = SC ? ld_sc1(p) : *p;
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int rr = (tid >> 6) + 4 * q, cc = tid & 63;
    dst[rr * DS + cc] = (rr < rows && cc < cols) ? v[q] : T(0);
  }
}

template <typename T, bool SC>
__device__ __forceinline__ void fetch_tile(T (&v)[16], const T* src, int64_t ld, int rows, int cols) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int rr = (tid >> 6) + 4 * q, cc = tid & 63;
    const T* p = &src[(int64_t)(rr < rows ? rr : 0) * ld + (cc < cols ? cc : 0)];
    v[q] = SC ? ld_sc1(p) : *p;
  }
}
template <typename T>
__device__ __forceinline__ void put_tile(T* dst, const T (&v)[16], int rows, int cols) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int rr = (tid >> 6) + 4 * q, cc = tid & 63;
    dst[rr * DS + cc] = (rr < rows && cc < cols) ? v[q] : T(0);
  }
}

// acc += W_prev[rows, 0:bop) L_prev[qrows, 0:bop)^T: the look-ahead update of
// one 64 x 64 tile with the previous outer panel (W_prev rows at Wr, ld ldw;
// L_prev rows at Lr, ld ld; both written by earlier launches), 64-deep
// chunks staged through As / Bs with the next chunk's loads in flight.
template <typename T>
__device__ __forceinline__ void prev_update(typename Mfma<T>::acc_t (&acc)[4], const T* Wr, int64_t ldw, const T* Lr,
                                            int64_t ld, int rows, int qrows, int bop, T* As, T* Bs) {
  T va[16], vb[16];
  fetch_tile<T, false>(va, Wr, ldw, rows, bop < 64 ? bop : 64);
  fetch_tile<T, false>(vb, Lr, ld, qrows, bop < 64 ? bop : 64);
  for (int kk = 0; kk < bop; kk += 64) {
    const int kw = bop - kk < 64 ? bop - kk : 64;
    __syncthreads();  // previous chunk's reads of As / Bs done
    put_tile<T>(As, va, rows, kw);
    put_tile<T>(Bs, vb, qrows, kw);
    __syncthreads();
    if (kk + 64 < bop) {
      const int kn = bop - kk - 64 < 64 ? bop - kk - 64 : 64;
      fetch_tile<T, false>(va, Wr + kk + 64, ldw, rows, kn);
      fetch_tile<T, false>(vb, Lr + kk + 64, ld, qrows, kn);
    }
    mma_tile<T, false>(As, [&](int r, int k) { return Bs[r * DS + k]; }, acc);
  }
  __syncthreads();
}

// accumulator-layout tile <-> global (lower part of a diagonal tile when DIAG)
template <typename T, bool SC, bool DIAGT>
__device__ __forceinline__ void load_acc(typename Mfma<T>::acc_t (&acc)[4], const T* src, int64_t ld, int rows,
                                         int cols) {
  typedef Mfma<T> MF;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int col = 16 * n + (lane & 15);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row = 16 * wave + MF::row(lane, g);
      const bool in = row < rows && col < cols && (!DIAGT || col <= row);
      const T* p = &src[(int64_t)(in ? row : 0) * ld + (in ? col : 0)];
      acc[n][g] = in ? (SC ? ld_sc1(p) : *p) : T(0);
    }
  }
}
template <typename T, bool SC, bool DIAGT>
__device__ __forceinline__ void store_acc(const typename Mfma<T>::acc_t (&acc)[4], T* dst, int64_t ld, int rows,
                                          int cols) {
  typedef Mfma<T> MF;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int col = 16 * n + (lane & 15);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row = 16 * wave + MF::row(lane, g);
      if (row < rows && col < cols && (!DIAGT || col <= row)) {
        if (SC) st_sc1(&dst[(int64_t)row * ld + col], acc[n][g]);
        else dst[(int64_t)row * ld + col] = acc[n][g];
      }
    }
  }
}
// accumulator-layout tile -> LDS (this wave's rows)
template <typename T>
__device__ __forceinline__ void put_acc(T* dst, const typename Mfma<T>::acc_t (&acc)[4]) {
  typedef Mfma<T> MF;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int g = 0; g < 4; ++g) dst[(16 * wave + MF::row(lane, g)) * DS + 16 * n + (lane & 15)] = acc[n][g];
}
template <typename T>
__device__ __forceinline__ void zero_acc(typename Mfma<T>::acc_t (&acc)[4]) {
#pragma unroll
  for (int n = 0; n < 4; ++n) acc[n] = (typename Mfma<T>::acc_t){T(0), T(0), T(0), T(0)};
}
}  // namespace

// ---------------------------------------------------------------------------
// One outer panel as ONE kernel launched twice -- on the chain stream (nchain
// workgroups) and on the rows stream after the look-ahead strip update of the
// rows below (nchain + nrows workgroups) -- with the roles handed out by two
// ticket counters:
//   chain tickets (area[OP_TICKET], both launches): [0, nchain) are the chain
//     roles: 0 = the CHAIN, 1 .. nb-1 = region HELPERS, nb .. = TILE WORKERS;
//     a workgroup that draws a later chain ticket takes no chain role;
//   rows tickets (area[OP_TICKET + 1], rows launch only): [0, nrows) = the
//     ROWS roles, one per 64 rows below the diagonal region.
// Whichever launch is dispatched first can hold every chain role, so no
// workgroup ever waits for one that has not been dispatched: the panel
// completes even when the two launches run one after the other in either
// order (rocprofv3 --pmc serializes dispatches; a device shared with other
// work may too).  The rows roles stay in the launch ordered after the strip
// update: they read its output, and a workgroup of the chain launch may have
// started before that output existed (its L2 could then serve stale lines --
// measured: shared rows tickets gave wrong C5 factors).
//
// T = float: the fp32 factor of the mixed-precision path (f32 MFMA TRSMs and
// strip pieces; the 64 x 64 diagonal blocks are factored in fp64 and stored
// in fp32).
// amdgpu_waves_per_eu(2): <= 256 registers per lane (VGPR + AGPR), so a
// panel workgroup fits beside a trailing-GEMM workgroup (64 per lane at 4
// waves per SIMD) -- with more it waits for a CU with no GEMM at all
namespace {
template <typename T>
struct PanelArgs {
  T* K;
  int64_t ld;
  int N, k0, c1;
  T* D;
  T* Lb0;
  T* Wp;
  int ldw;
  int* info;
  unsigned* area;
  unsigned* err;
  int inject;
  const T* Wprev;  // previous panel's W (nullptr: no look-ahead update in this launch pair)
  int kprev, boprev;
  const T* pre00_in;  // this panel's block (0, 0) update, accumulated by the previous rows role 0
  T* pre00_out;       // the next panel's, accumulated by rows role 0
  int nchain;         // chain-role tickets
  int nrows;          // rows-role tickets
};

// ---- the chain roles (tickets < nchain)
template <typename T>
__device__ __forceinline__ void chain_roles(const PanelArgs<T>& a, int t, double* smem, unsigned* sh_ok) {
  typedef Mfma<T> MF;
  typedef typename MF::acc_t acc_t;
  T* const K = a.K;
  const int64_t ld = a.ld;
  const int k0 = a.k0, ldw = a.ldw;
  T* const D = a.D;
  T* const Lb0 = a.Lb0;
  T* const Wp = a.Wp;
  unsigned* const area = a.area;
  unsigned* const err = a.err;
  const T* const Wprev = a.Wprev;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ce = a.c1 < a.N ? a.c1 : a.N;
  const int nb = (ce - k0 + 63) / 64;
  double* M = smem;
  double* X = smem + 64 * DS;
  double* dsh = smem + 2 * 64 * DS;  // 64 doubles (diag64_body's pivots)
  auto bsz = [&](int j) { return ce - (k0 + 64 * j) < 64 ? ce - (k0 + 64 * j) : 64; };

  if (t == 0) {
    // ================================================================ CHAIN
    if (Wprev) {  // block (0, 0) with the previous panel's update, straight into M
      acc_t own[4];
      if (a.pre00_in) {
        // accumulated by the previous panel's rows role 0 (the same MFMA
        // order as prev_update), so this role starts with the diagonal factor
        load_acc<T, false, false>(own, a.pre00_in, 64, 64, 64);
      } else {
        zero_acc<T>(own);
        prev_update<T>(own, Wprev + (int64_t)k0 * ldw, ldw, K + (int64_t)k0 * ld + a.kprev, ld, bsz(0), bsz(0),
                       a.boprev, reinterpret_cast<T*>(M), reinterpret_cast<T*>(X));
      }
      acc_t a0[4];
      load_acc<T, false, true>(a0, K + (int64_t)k0 * ld + k0, ld, bsz(0), bsz(0));
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int col = 16 * n + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = 16 * wave + MF::row(lane, g);
          M[row * DS + col] = (row < bsz(0) && col <= row) ? (double)(a0[n][g] - own[n][g]) : (row == col ? 1.0 : 0.0);
        }
      }
    }
    for (int j = 0; j < nb; ++j) {
      const int j0 = k0 + 64 * j, bj = bsz(j);
      CSTAMP(j0 / 64, 0);
      T* Lb = Lb0 + (int64_t)j * 64 * 64;
      // ---- block row c = j + 1: (c, j) and (c, c) from helper c.  Once the
      // diagonal block is final in LDS and before its write-back, one load
      // per 128-byte line of both tiles pulls them into this XCD's L2 (the
      // helper stored them write-through): the operand loads after the
      // write-back then hit L2 instead of paying the HBM latency on the chain
      const bool more = j + 1 < nb;
      const int c = j + 1, r0 = k0 + 64 * c, rows = more ? bsz(c) : 0;
      bool ok = true;
      T pf[2] = {T(0), T(0)};
      auto next_prefetch = [&]() {
        if (!more) return;
        ok = wait_flag(&area[OP_READY + c], err, sh_ok);  // (uniform)
        CSTAMP(j0 / 64, 1);
        if (!ok) return;
        const int line = threadIdx.x, rr = line >> 2, cc = (line & 3) * (128 / (int)sizeof(T));
        if (rr < rows) {
          pf[0] = ld_sc1(&K[(int64_t)(r0 + rr) * ld + j0 + (cc < 64 ? cc : 0)]);
          pf[1] = ld_sc1(&K[(int64_t)(r0 + rr) * ld + r0 + (cc <= rr ? cc : 0)]);
        }
      };
      if (j == 0 && !Wprev)
        diag64_body<true, false, T, false>(K, ld, j0, bj, D, Lb, a.info, M, X, dsh, nullptr, next_prefetch);
      else
        diag64_body<true, false, T, true>(K, ld, j0, bj, D, Lb, a.info, M, X, dsh, nullptr, next_prefetch);
      CSTAMP(j0 / 64, 2);
      if (!more) {
        if (!(a.inject && j == 0)) publish(&area[OP_DIAG + j]);
        break;
      }
      if (!ok) return;
      asm volatile("" ::"v"(pf[0]), "v"(pf[1]));  // the prefetches stay live (not eliminated) until here
      // A(c, j) into M (free: L_jj is in K), the own block (c, c) into registers
      stage_tile<T, true>(reinterpret_cast<T*>(M), K + (int64_t)r0 * ld + j0, ld, rows, 64);
      acc_t own[4];
      load_acc<T, true, true>(own, K + (int64_t)r0 * ld + r0, ld, rows, rows);
      // DIAG[j] after these loads: the diagonal block's write-back drains beside
      // them instead of on the chain (nothing this workgroup waits for needs
      // DIAG[j]: helper c only uses blocks <= c - 2).  inject: timeout tests only
      if (!(a.inject && j == 0)) publish(&area[OP_DIAG + j]);
      CSTAMP(j0 / 64, 3);
      T rd[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) rd[n] = T(1) / (T)dsh[16 * n + (lane & 15)];
      __syncthreads();
      // TRSM: T = A(c, j) X_jj^T with X lower triangular (its upper part in
      // LDS is not meaningful: masked)
      acc_t acc[4];
      zero_acc<T>(acc);
      mma_tile_lower<T>(reinterpret_cast<const T*>(M), [&](int r, int k) { return k <= r ? (T)X[r * DS + k] : T(0); },
                        acc);
      __syncthreads();  // M and X reads done
      CSTAMP(j0 / 64, 4);
      T* Lrow = K + (int64_t)r0 * ld + j0;
      T* Wrow = Wp + (int64_t)r0 * ldw + 64 * j;
      acc_t lacc[4];
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) lacc[n][g] = acc[n][g] * rd[n];
      store_acc<T, false, false>(lacc, Lrow, ld, rows, 64);
      store_acc<T, true, false>(acc, Wrow, ldw, rows, 64);
      // own update (c, c) -= L(c, j) W(c, j)^T: L into X, W into M (both free:
      // L_jj is in K, X_jj no longer needed)
      T* Lx = reinterpret_cast<T*>(X);
      T* Wm = reinterpret_cast<T*>(M);
      put_acc<T>(Lx, lacc);
      put_acc<T>(Wm, acc);
      __syncthreads();
      mma_tile<T, true>(Lx, [&](int r, int k) { return Wm[r * DS + k]; }, own);
      // W(c, j) for the helpers' and the rows roles' strips: published after
      // the update, so the stores drain beside its MFMAs (publish's barrier
      // also ends every wave's reads of M and X)
      publish(&area[OP_REG + j * OP_NBMAX + c]);
      CSTAMP(j0 / 64, 5);
      // the next diagonal block, straight into diag64_body's image
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int col = 16 * n + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = 16 * wave + MF::row(lane, g);
          M[row * DS + col] = (row < rows && col <= row) ? (double)own[n][g] : (row == col ? 1.0 : 0.0);
        }
      }
      // (diag64_body's first barrier orders these stores before its reads)
    }
    return;
  }
  if (t >= nb) {
    // ============================================================ TILE WORKER
    // region block (c, q), 1 <= c < nb, q <= c: the look-ahead update with the
    // previous panel, stored write-through, then TILE[c][q]
    int w = t - nb, c = 1;
    while (w > c) {
      w -= c + 1;
      ++c;
    }
    const int q = w, r0 = k0 + 64 * c, q0 = k0 + 64 * q, rows = bsz(c), qrows = bsz(q);
    acc_t upd[4], tile[4];
    zero_acc<T>(upd);
    prev_update<T>(upd, Wprev + (int64_t)r0 * ldw, ldw, K + (int64_t)q0 * ld + a.kprev, ld, rows, qrows, a.boprev,
                   reinterpret_cast<T*>(M), reinterpret_cast<T*>(X));
    if (q == c) load_acc<T, false, true>(tile, K + (int64_t)r0 * ld + q0, ld, rows, rows);
    else load_acc<T, false, false>(tile, K + (int64_t)r0 * ld + q0, ld, rows, qrows);
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) tile[n][g] = tile[n][g] - upd[n][g];
    if (q == c) store_acc<T, true, true>(tile, K + (int64_t)r0 * ld + q0, ld, rows, rows);
    else store_acc<T, true, false>(tile, K + (int64_t)r0 * ld + q0, ld, rows, qrows);
    publish(&area[OP_TILE + c * OP_NBMAX + q]);
    return;
  }
  // ================================================================= HELPER
  const int c = t, r0 = k0 + 64 * c, rows = bsz(c);
  T* As = reinterpret_cast<T*>(M);  // L(c, j) rows
  T* Bs = reinterpret_cast<T*>(X);  // L_jj^{-1}, then W pieces
  if (Wprev) {  // this row of region blocks, updated with the previous panel by the tile workers
    for (int q = 0; q <= c; ++q)
      if (!wait_flag(&area[OP_TILE + c * OP_NBMAX + q], err, sh_ok)) return;
  }
  for (int j = 0; j + 2 <= c; ++j) {
    const int j0 = k0 + 64 * j;
    T* Lb = Lb0 + (int64_t)j * 64 * 64;
    if (j || Wprev) stage_tile<T, true>(As, K + (int64_t)r0 * ld + j0, ld, rows, 64);
    else stage_tile<T, false>(As, K + (int64_t)r0 * ld + j0, ld, rows, 64);
    if (!wait_flag(&area[OP_DIAG + j], err, sh_ok)) return;
    stage_tile<T, true>(Bs, Lb, 64, 64, 64);
    T rd[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) rd[n] = T(1) / ld_sc1(&D[j0 + 16 * n + (lane & 15)]);
    __syncthreads();
    acc_t acc[4];
    zero_acc<T>(acc);
    mma_tile_lower<T>(As, [&](int r, int k) { return Bs[r * DS + k]; }, acc);  // L_jj^{-1}: lower
    __syncthreads();
    acc_t lacc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) lacc[n][g] = acc[n][g] * rd[n];
    store_acc<T, false, false>(lacc, K + (int64_t)r0 * ld + j0, ld, rows, 64);
    store_acc<T, true, false>(acc, Wp + (int64_t)r0 * ldw + 64 * j, ldw, rows, 64);
    publish(&area[OP_REG + j * OP_NBMAX + c]);
    put_acc<T>(As, lacc);
    // strips: (c, q) -= L(c, j) W(q, j)^T, q = j+1 .. c
    for (int q = j + 1; q <= c; ++q) {
      const int q0 = k0 + 64 * q, qrows = bsz(q);
      if (q == c) {
        put_acc<T>(Bs, acc);
      } else {
        if (!wait_flag(&area[OP_REG + j * OP_NBMAX + q], err, sh_ok)) return;
        stage_tile<T, true>(Bs, Wp + (int64_t)q0 * ldw + 64 * j, ldw, qrows, 64);
      }
      acc_t tile[4];
      if (q == c) load_acc<T, true, true>(tile, K + (int64_t)r0 * ld + q0, ld, rows, rows);
      else load_acc<T, true, false>(tile, K + (int64_t)r0 * ld + q0, ld, rows, qrows);
      __syncthreads();
      mma_tile<T, true>(As, [&](int r, int k) { return Bs[r * DS + k]; }, tile);
      if (q == c) store_acc<T, true, true>(tile, K + (int64_t)r0 * ld + q0, ld, rows, rows);
      else store_acc<T, true, false>(tile, K + (int64_t)r0 * ld + q0, ld, rows, qrows);
      __syncthreads();  // Bs reused by the next piece
    }
  }
  publish(&area[OP_READY + c]);
  HSTAMP(r0 / 64, 0);
}

// ---- a rows role (rows ticket r): the 64 rows from ce + 64 r.  Every
// operand another role of this panel produced is read with agent-scope loads
// (the producer may be in the other launch).  rows_prev: first the
// look-ahead update of these rows with the PREVIOUS panel, A[rows, panel] -=
// W_prev[rows] L_prev[panel rows]^T (the fused factor runs it as a strip GEMM
// on the rows stream instead).
template <typename T>
__device__ __forceinline__ void rows_role(const PanelArgs<T>& a, int r, bool rows_prev, double* smem,
                                          unsigned* sh_ok) {
  typedef typename Mfma<T>::acc_t acc_t;
  T* const K = a.K;
  const int64_t ld = a.ld;
  const int k0 = a.k0, N = a.N, ldw = a.ldw;
  const int lane = threadIdx.x & 63;
  const int ce = a.c1 < N ? a.c1 : N;
  const int nb = (ce - k0 + 63) / 64;
  const int row0 = ce + 64 * r;
  const int rows = N - row0 < 64 ? N - row0 : 64;
  auto bsz = [&](int j) { return ce - (k0 + 64 * j) < 64 ? ce - (k0 + 64 * j) : 64; };
  T* As = reinterpret_cast<T*>(smem);
  T* Bs = reinterpret_cast<T*>(smem + 64 * DS);
  T* Krow = K + (int64_t)row0 * ld;
  if (rows_prev) {
    for (int q = 0; q < nb; ++q) {
      const int q0 = k0 + 64 * q, qrows = bsz(q);
      acc_t acc[4], tile[4];
      zero_acc<T>(acc);
      prev_update<T>(acc, a.Wprev + (int64_t)row0 * ldw, ldw, K + (int64_t)q0 * ld + a.kprev, ld, rows, qrows,
                     a.boprev, As, Bs);
      load_acc<T, true, false>(tile, Krow + q0, ld, rows, qrows);
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) tile[n][g] = tile[n][g] - acc[n][g];
      store_acc<T, false, false>(tile, Krow + q0, ld, rows, qrows);
    }
  }
  // ---- TRSMs and strips of this chunk's rows.  Role 0 (the next panel's
  // first 64 rows) also accumulates that panel's block (0, 0) look-ahead
  // update W(rows, j) L(rows, j)^T over j -- exactly the chunks prev_update
  // would sum in the next chain role -- and leaves it in pre00_out.
  if (r == 0) HSTAMP(k0 / 64, 1);
  T* const p00 = r == 0 ? a.pre00_out : nullptr;
  acc_t a00[4];
  zero_acc<T>(a00);
  bool ok = true;
  for (int j = 0; j < nb && ok; ++j) {
    const int j0 = k0 + 64 * j, bj = bsz(j);
    const T* Lb = a.Lb0 + (int64_t)j * 64 * 64;
    __syncthreads();  // previous block's strip finished reading As / Bs
    stage_tile<T, true>(As, Krow + j0, ld, rows, bj);
    if (!(ok = wait_flag(&a.area[OP_DIAG + j], a.err, sh_ok))) break;
    stage_tile<T, true>(Bs, Lb, 64, 64, 64);
    T rd[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = 16 * n + (lane & 15);
      rd[n] = col < bj ? T(1) / ld_sc1(&a.D[j0 + col]) : T(0);
    }
    __syncthreads();
    acc_t acc[4];
    zero_acc<T>(acc);
    mma_tile_lower<T>(As, [&](int rr, int k) { return Bs[rr * DS + k]; }, acc);  // L_jj^{-1}: lower
    __syncthreads();
    acc_t lacc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) lacc[n][g] = acc[n][g] * rd[n];
    store_acc<T, false, false>(lacc, Krow + j0, ld, rows, bj);
    store_acc<T, false, false>(acc, a.Wp + (int64_t)row0 * ldw + 64 * j, ldw, rows, bj);
    put_acc<T>(As, lacc);
    if (p00) {  // a00 += W(rows, j) L(rows, j)^T (W staged in Bs, L in As)
      put_acc<T>(Bs, acc);
      __syncthreads();
      mma_tile<T, false>(Bs, [&](int rr, int k) { return As[rr * DS + k]; }, a00);
      __syncthreads();  // Bs is reused by the strips
    }
    // strips: (rows, q) -= L(rows, j) W(q, j)^T, q = j+1 .. nb-1
    for (int q = j + 1; q < nb; ++q) {
      const int q0 = k0 + 64 * q, qrows = bsz(q);
      if (!(ok = wait_flag(&a.area[OP_REG + j * OP_NBMAX + q], a.err, sh_ok))) break;  // (its barrier also frees Bs)
      stage_tile<T, true>(Bs, a.Wp + (int64_t)q0 * ldw + 64 * j, ldw, qrows, bj);
      acc_t tile[4];
      load_acc<T, true, false>(tile, Krow + q0, ld, rows, qrows);
      __syncthreads();
      mma_tile<T, true>(As, [&](int rr, int k) { return Bs[rr * DS + k]; }, tile);
      store_acc<T, false, false>(tile, Krow + q0, ld, rows, qrows);
      __syncthreads();
    }
  }
  if (p00 && ok) store_acc<T, false, false>(a00, p00, 64, 64, 64);  // consumed by a later launch
  if (r == 0) HSTAMP(k0 / 64, 2);
}
}  // namespace

template <typename T>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void panel_kernel(PanelArgs<T> a,
                                                                                           int rows_launch, int rows_prev) {
  // M, X: diag64_body's images (66.5 KB: a panel workgroup fits the LDS one
  // trailing-GEMM workgroup leaves free, so it is never starved of a CU)
  __shared__ __attribute__((aligned(16))) double smem[2 * 64 * DS + 64];
  __shared__ unsigned sh_ticket, sh_ok;
  if (threadIdx.x == 0) {
    unsigned t = atomicAdd(&a.area[OP_TICKET], 1u);  // a chain role, while any is left
    if (t >= (unsigned)a.nchain) t = rows_launch ? a.nchain + atomicAdd(&a.area[OP_TICKET + 1], 1u) : ~0u;
    sh_ticket = t;
  }
  __syncthreads();
  const unsigned tu = sh_ticket;
  if (tu == ~0u) return;
  const int t = (int)tu;
  if (t == 0) HSTAMP(a.k0 / 64 + 1, 3);  // the chain role's workgroup starts
  if (t == a.nchain) HSTAMP(a.k0 / 64 + 2, 3);  // the first rows role starts
  if (t < a.nchain) {
    // s_setprio 3: the chain roles' waves win issue arbitration (matrix pipe
    // included) against the GEMM waves that share the CU
    __builtin_amdgcn_s_setprio(3);
    chain_roles<T>(a, t, smem, &sh_ok);
  } else if (t < a.nchain + a.nrows) {
    rows_role<T>(a, t - a.nchain, rows_prev != 0, smem, &sh_ok);
  }
}

// ---------------------------------------------------------------------------
template <typename T>
static hipError_t panel_launch_t(T* K, int64_t ld, int N, int k0, int bo, T* D, T* Lb0, T* Wp, int ldw,
                                 const T* pre00_in, T* pre00_out, int* info,
                                 unsigned* area, unsigned* err, const T* Wprev, int kprev, int boprev, bool rows_prev,
                                 hipStream_t st_chain, hipStream_t st_rows) {
  if (bo <= 0 || bo > IPMZ_NBO_MAX || k0 + bo > N) return hipErrorInvalidValue;
  const int ce = k0 + bo;
  const int nb = (bo + 63) / 64;
  PanelArgs<T> a;
  a.K = K;
  a.ld = ld;
  a.N = N;
  a.k0 = k0;
  a.c1 = ce;
  a.D = D;
  a.Lb0 = Lb0;
  a.Wp = Wp;
  a.ldw = ldw;
  a.info = info;
  a.area = area;
  a.err = err;
  a.inject = debug_inject_mask() & IPMZ_INJECT_PANEL;
  a.Wprev = Wprev;
  a.kprev = kprev;
  a.boprev = boprev;
  a.pre00_in = Wprev ? pre00_in : nullptr;
  a.pre00_out = pre00_out;
  // chain + nb - 1 helpers (+ one tile worker per region block below the
  // diagonal block (0, 0) when the look-ahead update is applied here)
  a.nchain = nb + (Wprev ? nb * (nb + 1) / 2 - 1 : 0);
  a.nrows = ce < N ? (N - ce + 63) / 64 : 0;
  hipLaunchKernelGGL(panel_kernel<T>, dim3(a.nchain), dim3(256), 0, st_chain, a, 0, rows_prev ? 1 : 0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || a.nrows == 0) return e;
  // the rows launch: every chain role and every rows role, should it run first
  hipLaunchKernelGGL(panel_kernel<T>, dim3(a.nchain + a.nrows), dim3(256), 0, st_rows, a, 1, rows_prev ? 1 : 0);
  return hipGetLastError();
}
hipError_t panel_factor(double* K, int64_t ld, int N, int k0, int bo, double* D, double* Lb0, double* Wp, int ldw,
                        const double* pre00_in, double* pre00_out, int* info, unsigned* area, unsigned* err,
                        const double* Wprev, int kprev, int boprev, bool rows_prev, hipStream_t st_chain,
                        hipStream_t st_rows) {
  return panel_launch_t<double>(K, ld, N, k0, bo, D, Lb0, Wp, ldw, pre00_in, pre00_out, info, area, err, Wprev, kprev,
                                boprev, rows_prev, st_chain, st_rows);
}
hipError_t panel_factor(float* K, int64_t ld, int N, int k0, int bo, float* D, float* Lb0, float* Wp, int ldw,
                        const float* pre00_in, float* pre00_out, int* info, unsigned* area, unsigned* err,
                        const float* Wprev, int kprev, int boprev, bool rows_prev, hipStream_t st_chain,
                        hipStream_t st_rows) {
  return panel_launch_t<float>(K, ld, N, k0, bo, D, Lb0, Wp, ldw, pre00_in, pre00_out, info, area, err, Wprev, kprev,
                               boprev, rows_prev, st_chain, st_rows);
}

}  // namespace ipmz
