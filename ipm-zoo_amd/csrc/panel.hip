// The panel path of the blocked LDL^T: for one outer panel (columns
// [k0, c1), nb <= 8 inner blocks of 64), the column loop of
// LinearSolvers::ldlt_decomposition (LinearSolvers.cpp:20-40) restricted to
// those columns, as roles that hand off by flags.  Two launches per panel --
// the CHAIN launch (panel_chain_kernel, 512 threads, on the chain stream) and
// the ROWS launch (panel_kernel, 256 threads, on the rows stream after the
// look-ahead strip update of the rows below) -- and every workgroup takes its
// role from ticket counters (the chain roles' shared by both launches; see
// panel_kernel for why that cannot deadlock):
//
//   chain roles (the panel's diagonal region, first updated with the previous
//   panel; s_setprio 3):
//     ticket 0 = the CHAIN: for every inner block j, factor the 64 x 64
//       diagonal block (diag64_body), publish DIAG[j], the TRSM of the next
//       region block (j+1, j) and that block's own diagonal update; the
//       result IS the next diagonal block.  The whole critical path of the
//       panel lives on one CU.  chain4 (4 waves, the default): one step
//       after the other.  chain8 (the 512-thread chain launch, debug bit
//       IPMZ_DEBUG_CHAIN8): waves 0-3 factor the diagonal block, waves 4-7
//       form the TRSM and the next diagonal block in its shadow, column block
//       by column block as the pivots and the rows of L_jj^{-1} become final
//       -- measured slower so far (27 vs 24 us per 64-column block at
//       N = 2560): it waits for helper c's READY, which follows the chain's
//       own REG[c-2][c-1] by ~11 us of hand-offs.
//     tickets nb.. = TILE WORKERS: one region block (c, q), c >= 1, each,
//       updated with the previous panel (flag TILE[c][q]); the chain updates
//       block (0, 0) itself, straight into its LDS image.
//     ticket c < nb = region HELPER c (rows of block c): the TRSMs of its
//       blocks j <= c - 2 and their strip updates, then READY[c]: its blocks
//       (c, c-1) and (c, c) carry every contribution but block c-1's, which
//       the chain applies itself.
//   rows roles (rows launch; one per 64 rows below the region): for every j:
//     TRSM with L_jj^{-1} (waits DIAG[j]), L = T / D, W = T, and the strip
//     pieces A[rows, q] -= L W[q, j]^T (waits REG[j][q]).
//
// Every role computes each element with the same operations in the same order
// in both of its forms (the 8-wave helpers and tile workers split a tile's
// column blocks over two waves per row block; chain8's bulk waves run chain4's
// MFMA sequences per column block), so the factor is bitwise the same
// whichever launch holds a role (tests/test_gpu_panel_forms.py, debug bits
// IPMZ_DEBUG_CHAIN8 / IPMZ_DEBUG_ROWS_CHAIN).
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
// seen, 2 diag done, 3 operands loaded (chain4) / first transition barrier
// (chain8), 4 TRSM done (chain4), 5 next diagonal block formed; helpers:
// READY[c] published; rows role 0: start, end; launches: first workgroup
// start per launch.
__device__ unsigned long long g_cstamp[IPMZ_CHAIN_STAMP_BLOCKS][8];
__device__ unsigned long long g_hstamp[IPMZ_CHAIN_STAMP_BLOCKS][4];
#ifdef IPMZ_CHAIN_STAMPS
#define CSTAMP_T(t0, jb, i) \
  if (threadIdx.x == (t0) && (jb) < IPMZ_CHAIN_STAMP_BLOCKS) g_cstamp[jb][i] = __builtin_amdgcn_s_memrealtime()
#define HSTAMP(jb, i) \
  if (threadIdx.x == 0 && (jb) < IPMZ_CHAIN_STAMP_BLOCKS) g_hstamp[jb][i] = __builtin_amdgcn_s_memrealtime()
#else
#define CSTAMP_T(t0, jb, i)
#define HSTAMP(jb, i)
#endif
#define CSTAMP(jb, i) CSTAMP_T(0, jb, i)
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

template <typename T>
using Acc = typename Mfma<T>::acc_t;

// The lane's place in a 64 x 64 tile in MFMA accumulator layout spread over
// NW waves: rows 16 wr + row(lane, g), column blocks n0 .. n0 + NN - 1
// (columns 16 n + (lane & 15)).  NW = 4: wave w holds row block w, every
// column block (the layout of waves 4..7 of chain8 as well: wr = w & 3);
// NW = 8: waves w and w + 4 share row block w & 3, the lower / upper two
// column blocks.  tid: the caller's thread index, laundered per loop
// iteration so the lane-dependent addresses are not hoisted (and spilled)
// across the block loops.
template <int NW>
struct TMap {
  static constexpr int NN = 16 / NW;
  int lane, wr, n0;
  __device__ __forceinline__ explicit TMap(int tid)
      : lane(tid & 63),
        wr(__builtin_amdgcn_readfirstlane((tid >> 6) & 3)),
        n0(NW == 8 ? __builtin_amdgcn_readfirstlane(2 * ((tid >> 8) & 1)) : 0) {}
};
__device__ __forceinline__ int launder(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// acc[i] (+)= sgn * A[16 wr.., :] B[16 n.., :]^T over k in [0, 64), n = n0 + i:
// A, B row-major 64 x DS tiles in LDS (B read through bf: (row, k) -> T).
// Per element: the MFMAs of k = 4s .. 4s+3, s = 0..15, in order.
template <typename T, bool NEG, int NW, typename BF>
__device__ __forceinline__ void mma_tile(const TMap<NW>& m, const T* As, BF bf, Acc<T> (&acc)[TMap<NW>::NN]) {
  typedef Mfma<T> MF;
  const int arow = 16 * m.wr + (m.lane & 15);
#pragma unroll 4
  for (int s = 0; s < 16; ++s) {
    const int k = 4 * s + (m.lane >> 4);
    const T a = NEG ? -As[arow * DS + k] : As[arow * DS + k];
#pragma unroll
    for (int i = 0; i < TMap<NW>::NN; ++i) acc[i] = MF::mma(a, bf(16 * (m.n0 + i) + (m.lane & 15), k), acc[i]);
  }
}

// acc[i] += A[16 wr.., :] B[16 n.., :]^T for a LOWER-triangular B (the
// diagonal block's inverse): k-chunks past column block n's diagonal are zero
// and skipped (40 of 64 MFMAs per 4-wave tile), the diagonal chunk masked
// through bf.  The chain's TRSM step: 4.5 -> 2.5 us per block.
template <typename T, int NW, typename BF>
__device__ __forceinline__ void mma_tile_lower(const TMap<NW>& m, const T* As, BF bf, Acc<T> (&acc)[TMap<NW>::NN]) {
  typedef Mfma<T> MF;
  const int arow = 16 * m.wr + (m.lane & 15);
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int k = 4 * s + (m.lane >> 4);
    const T a = As[arow * DS + k];
#pragma unroll
    for (int i = 0; i < TMap<NW>::NN; ++i) {
      const int n = m.n0 + i;  // (wave-uniform)
      if (s < 4 * (n + 1)) acc[i] = MF::mma(a, bf(16 * n + (m.lane & 15), k), acc[i]);
    }
  }
}

// 64 x 64 tile of a row-major matrix (ld) into LDS (rows < rows, columns <
// cols; zeros elsewhere) by NW waves: 64 / NW loads in flight per thread.
// SC: agent-scope loads (data written earlier in this launch, possibly by
// another CU).
template <typename T, bool SC, int NW>
__device__ __forceinline__ void fetch_tile(int tid, T (&v)[64 / NW], const T* src, int64_t ld, int rows, int cols) {
  const int w = (tid >> 6) & (NW - 1), cc = tid & 63;
#pragma unroll
  for (int q = 0; q < 64 / NW; ++q) {
    const int rr = w + NW * q;
    const T* p = &src[(int64_t)(rr < rows ? rr : 0) * ld + (cc < cols ? cc : 0)];
    v[q] = SC ? ld_sc1(p) : *p;
  }
}
template <typename T, int NW>
__device__ __forceinline__ void put_tile(int tid, T* dst, const T (&v)[64 / NW], int rows, int cols) {
  const int w = (tid >> 6) & (NW - 1), cc = tid & 63;
#pragma unroll
  for (int q = 0; q < 64 / NW; ++q) {
    const int rr = w + NW * q;
    dst[rr * DS + cc] = (rr < rows && cc < cols) ? v[q] : T(0);
  }
}
template <typename T, bool SC, int NW>
__device__ __forceinline__ void stage_tile(int tid, T* dst, const T* src, int64_t ld, int rows, int cols) {
  T v[64 / NW];
  fetch_tile<T, SC, NW>(tid, v, src, ld, rows, cols);
  put_tile<T, NW>(tid, dst, v, rows, cols);
}

// acc += W_prev[rows, 0:bop) L_prev[qrows, 0:bop)^T: the look-ahead update of
// one 64 x 64 tile with the previous outer panel (W_prev rows at Wr, ld ldw;
// L_prev rows at Lr, ld ld; both written by earlier launches), 64-deep
// chunks staged through As / Bs with the next chunk's loads in flight.
template <typename T, int NW>
__device__ __forceinline__ void prev_update(int tid, Acc<T> (&acc)[TMap<NW>::NN], const T* Wr, int64_t ldw,
                                            const T* Lr, int64_t ld, int rows, int qrows, int bop, T* As, T* Bs) {
  const TMap<NW> m(tid);
  T va[64 / NW], vb[64 / NW];
  fetch_tile<T, false, NW>(tid, va, Wr, ldw, rows, bop < 64 ? bop : 64);
  fetch_tile<T, false, NW>(tid, vb, Lr, ld, qrows, bop < 64 ? bop : 64);
  for (int kk = 0; kk < bop; kk += 64) {
    const int kw = bop - kk < 64 ? bop - kk : 64;
    __syncthreads();  // previous chunk's reads of As / Bs done
    put_tile<T, NW>(tid, As, va, rows, kw);
    put_tile<T, NW>(tid, Bs, vb, qrows, kw);
    __syncthreads();
    if (kk + 64 < bop) {
      const int kn = bop - kk - 64 < 64 ? bop - kk - 64 : 64;
      fetch_tile<T, false, NW>(tid, va, Wr + kk + 64, ldw, rows, kn);
      fetch_tile<T, false, NW>(tid, vb, Lr + kk + 64, ld, qrows, kn);
    }
    mma_tile<T, false, NW>(m, As, [&](int r, int k) { return Bs[r * DS + k]; }, acc);
  }
  __syncthreads();
}

// accumulator-layout tile <-> global (lower part of a diagonal tile when DIAGT)
template <typename T, bool SC, bool DIAGT, int NW>
__device__ __forceinline__ void load_acc(const TMap<NW>& m, Acc<T> (&acc)[TMap<NW>::NN], const T* src, int64_t ld,
                                         int rows, int cols) {
  typedef Mfma<T> MF;
#pragma unroll
  for (int i = 0; i < TMap<NW>::NN; ++i) {
    const int col = 16 * (m.n0 + i) + (m.lane & 15);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row = 16 * m.wr + MF::row(m.lane, g);
      const bool in = row < rows && col < cols && (!DIAGT || col <= row);
      const T* p = &src[(int64_t)(in ? row : 0) * ld + (in ? col : 0)];
      acc[i][g] = in ? (SC ? ld_sc1(p) : *p) : T(0);
    }
  }
}
template <typename T, bool SC, bool DIAGT, int NW>
__device__ __forceinline__ void store_acc(const TMap<NW>& m, const Acc<T> (&acc)[TMap<NW>::NN], T* dst, int64_t ld,
                                          int rows, int cols) {
  typedef Mfma<T> MF;
#pragma unroll
  for (int i = 0; i < TMap<NW>::NN; ++i) {
    const int col = 16 * (m.n0 + i) + (m.lane & 15);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row = 16 * m.wr + MF::row(m.lane, g);
      if (row < rows && col < cols && (!DIAGT || col <= row)) {
        if (SC) st_sc1(&dst[(int64_t)row * ld + col], acc[i][g]);
        else dst[(int64_t)row * ld + col] = acc[i][g];
      }
    }
  }
}
// accumulator-layout tile -> LDS (this wave's rows and column blocks)
template <typename T, int NW>
__device__ __forceinline__ void put_acc(const TMap<NW>& m, T* dst, const Acc<T> (&acc)[TMap<NW>::NN]) {
  typedef Mfma<T> MF;
#pragma unroll
  for (int i = 0; i < TMap<NW>::NN; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      dst[(16 * m.wr + MF::row(m.lane, g)) * DS + 16 * (m.n0 + i) + (m.lane & 15)] = acc[i][g];
}
template <typename T, int NN>
__device__ __forceinline__ void zero_acc(Acc<T> (&acc)[NN]) {
#pragma unroll
  for (int i = 0; i < NN; ++i) acc[i] = (Acc<T>){T(0), T(0), T(0), T(0)};
}
// M (diag64_body's fp64 image, row stride DS) <- a - b for this lane's
// elements of the lower part of the first b0 rows, identity elsewhere
template <typename T, int NW>
__device__ __forceinline__ void put_diag_image(const TMap<NW>& m, double* M, const Acc<T> (&a)[TMap<NW>::NN],
                                               const Acc<T> (&b)[TMap<NW>::NN], int b0) {
  typedef Mfma<T> MF;
#pragma unroll
  for (int i = 0; i < TMap<NW>::NN; ++i) {
    const int col = 16 * (m.n0 + i) + (m.lane & 15);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row = 16 * m.wr + MF::row(m.lane, g);
      M[row * DS + col] = (row < b0 && col <= row) ? (double)(a[i][g] - b[i][g]) : (row == col ? 1.0 : 0.0);
    }
  }
}
}  // namespace

// ---------------------------------------------------------------------------
// One outer panel as TWO launches -- the chain launch (panel_chain_kernel,
// nchain workgroups of 512 threads) on the chain stream and the rows launch
// (panel_kernel, nchain + nrows workgroups of 256 threads) on the rows stream
// after the look-ahead strip update of the rows below -- with the roles handed
// out by two ticket counters:
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

template <typename T>
__device__ __forceinline__ int panel_nb(const PanelArgs<T>& a) {
  const int ce = a.c1 < a.N ? a.c1 : a.N;
  return (ce - a.k0 + 63) / 64;
}
template <typename T>
__device__ __forceinline__ int panel_bsz(const PanelArgs<T>& a, int j) {
  const int ce = a.c1 < a.N ? a.c1 : a.N;
  return ce - (a.k0 + 64 * j) < 64 ? ce - (a.k0 + 64 * j) : 64;
}

// Block (0, 0) of the panel with the previous panel's update, straight into
// diag64_body's image M (all NW waves)
template <typename T, int NW>
__device__ __forceinline__ void chain_block00(const PanelArgs<T>& a, double* M, double* X) {
  const int tid = launder((int)threadIdx.x);
  const TMap<NW> m(tid);
  const int k0 = a.k0, b0 = panel_bsz(a, 0);
  Acc<T> own[TMap<NW>::NN];
  if (a.pre00_in) {
    // accumulated by the previous panel's rows role 0 (the same MFMA order as
    // prev_update), so this role starts with the diagonal factor
    load_acc<T, false, false, NW>(m, own, a.pre00_in, 64, 64, 64);
  } else {
    zero_acc<T, TMap<NW>::NN>(own);
    prev_update<T, NW>(tid, own, a.Wprev + (int64_t)k0 * a.ldw, a.ldw, a.K + (int64_t)k0 * a.ld + a.kprev, a.ld, b0,
                       b0, a.boprev, reinterpret_cast<T*>(M), reinterpret_cast<T*>(X));
  }
  Acc<T> a0[TMap<NW>::NN];
  load_acc<T, false, true, NW>(m, a0, a.K + (int64_t)k0 * a.ld + k0, a.ld, b0, b0);
  put_diag_image<T, NW>(m, M, a0, own, b0);
  // (diag64_body's first barrier orders these stores before its reads)
}

// ---- CHAIN, 4 waves (a 256-thread workgroup of either launch): one step
// after the other, every step on the critical path
template <typename T>
__device__ __forceinline__ void chain4(const PanelArgs<T>& a, double* smem, unsigned* sh_ok) {
  T* const K = a.K;
  const int64_t ld = a.ld;
  const int k0 = a.k0, ldw = a.ldw;
  unsigned* const area = a.area;
  const int nb = panel_nb(a);
  double* M = smem;
  double* X = smem + 64 * DS;
  double* dsh = smem + 2 * 64 * DS;  // 64 doubles (diag64_body's pivots)
  if (a.Wprev) chain_block00<T, 4>(a, M, X);
  for (int j = 0; j < nb; ++j) {
    const int tid = launder((int)threadIdx.x), lane = tid & 63;
    const TMap<4> m(tid);
    const int j0 = k0 + 64 * j, bj = panel_bsz(a, j);
    CSTAMP(j0 / 64, 0);
    T* Lb = a.Lb0 + (int64_t)j * 64 * 64;
    // ---- block row c = j + 1: (c, j) and (c, c) from helper c.  Once the
    // diagonal block is final in LDS and before its write-back, one load
    // per 128-byte line of both tiles pulls them into this XCD's L2 (the
    // helper stored them write-through): the operand loads after the
    // write-back then hit L2 instead of paying the HBM latency on the chain
    const bool more = j + 1 < nb;
    const int c = j + 1, r0 = k0 + 64 * c, rows = more ? panel_bsz(a, c) : 0;
    bool ok = true;
    T pf[2] = {T(0), T(0)};
    auto next_prefetch = [&]() {
      if (!more) return;
      ok = wait_flag(&area[OP_READY + c], a.err, sh_ok);  // (uniform)
      CSTAMP(j0 / 64, 1);
      if (!ok) return;
      const int rr = tid >> 2, cc = (tid & 3) * (128 / (int)sizeof(T));
      if (rr < rows) {
        pf[0] = ld_sc1(&K[(int64_t)(r0 + rr) * ld + j0 + (cc < 64 ? cc : 0)]);
        pf[1] = ld_sc1(&K[(int64_t)(r0 + rr) * ld + r0 + (cc <= rr ? cc : 0)]);
      }
    };
    if (j == 0 && !a.Wprev)
      diag64_body<true, false, T, false>(K, ld, j0, bj, a.D, Lb, a.info, M, X, dsh, nullptr, next_prefetch, nullptr,
                                         tid);
    else
      diag64_body<true, false, T, true>(K, ld, j0, bj, a.D, Lb, a.info, M, X, dsh, nullptr, next_prefetch, nullptr,
                                        tid);
    CSTAMP(j0 / 64, 2);
    if (!more) {
      if (!(a.inject && j == 0)) publish(&area[OP_DIAG + j]);
      break;
    }
    if (!ok) return;
    asm volatile("" ::"v"(pf[0]), "v"(pf[1]));  // the prefetches stay live (not eliminated) until here
    // A(c, j) into M (free: L_jj is in K), the own block (c, c) into registers
    stage_tile<T, true, 4>(tid, reinterpret_cast<T*>(M), K + (int64_t)r0 * ld + j0, ld, rows, 64);
    Acc<T> own[4];
    load_acc<T, true, true, 4>(m, own, K + (int64_t)r0 * ld + r0, ld, rows, rows);
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
    Acc<T> acc[4];
    zero_acc<T, 4>(acc);
    mma_tile_lower<T, 4>(m, reinterpret_cast<const T*>(M),
                         [&](int r, int k) { return k <= r ? (T)X[r * DS + k] : T(0); }, acc);
    __syncthreads();  // M and X reads done
    CSTAMP(j0 / 64, 4);
    T* Lrow = K + (int64_t)r0 * ld + j0;
    T* Wrow = a.Wp + (int64_t)r0 * ldw + 64 * j;
    Acc<T> lacc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) lacc[n][g] = acc[n][g] * rd[n];
    store_acc<T, false, false, 4>(m, lacc, Lrow, ld, rows, 64);
    store_acc<T, true, false, 4>(m, acc, Wrow, ldw, rows, 64);
    // own update (c, c) -= L(c, j) W(c, j)^T: L into X, W into M (both free:
    // L_jj is in K, X_jj no longer needed)
    T* Lx = reinterpret_cast<T*>(X);
    T* Wm = reinterpret_cast<T*>(M);
    put_acc<T, 4>(m, Lx, lacc);
    put_acc<T, 4>(m, Wm, acc);
    __syncthreads();
    mma_tile<T, true, 4>(m, Lx, [&](int r, int k) { return Wm[r * DS + k]; }, own);
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
        const int row = 16 * m.wr + Mfma<T>::row(lane, g);
        M[row * DS + col] = (row < rows && col <= row) ? (double)own[n][g] : (row == col ? 1.0 : 0.0);
      }
    }
    // (diag64_body's first barrier orders these stores before its reads)
  }
}

// ---- CHAIN, 8 waves (the chain launch's 512-thread workgroup).  Waves 0-3
// (chain group) only factor diagonal blocks: diag64_body with its write-back,
// then two transition barriers.  Waves 4-7 (bulk group, chain4's tile layout:
// wave 4 + w holds rows 16 w.. of every tile) form, in the shadow of diag(j),
// what chain4 runs after it -- T = A(c, j) X_jj^T, L = T / D, and the own
// update (c, c) -= L W^T with W = T -- column block by column block as the
// pivots D_n (after column pass n) and the rows X_n of L_jj^{-1} (after the
// inverse tiles of block row n) become final; each block's values come from
// the same MFMA sequence as in chain4.  The window's barriers are diag64_body's
// ten (intervals I1 .. I10) plus T1 / T2:
//   I2 (first column pass): drain the previous block's stores;
//   after #2: publish DIAG[j-1], REG[j-1][j] (stored in the last transition);
//   I6 (column pass 2): wait READY[c], load A(c, j) (TRSM operand) and (c, c);
//   I8 (column pass 3): TRSM column blocks 0, 1 -> Tb (the T tile in LDS);
//   I9: own update with k blocks 0, 1; TRSM column block 2 -> Tb;
//   I10: own update with k block 2;
//   transition (after #10, beside the chain group's write-back of L_jj,
//   L_jj^{-1}, D): TRSM column block 3 -> Tb; T1; own update with k block 3,
//   the stores of L(c, j) and W(c, j) (published after #2 of the next
//   window), the next diagonal block into M; T2.
// So the critical path per block is the diagonal factor, the last column
// block's TRSM and the last k block of the own update.  LDS: M, X, dsh, Tb and
// its reciprocal pivots rdb (100 KB: the workgroup fits beside one
// trailing-GEMM workgroup's 48 KB).
template <typename T>
__device__ __forceinline__ void chain8(const PanelArgs<T>& a, double* smem) {
  typedef Mfma<T> MF;
  T* const K = a.K;
  const int64_t ld = a.ld;
  const int k0 = a.k0, ldw = a.ldw;
  unsigned* const area = a.area;
  const int nb = panel_nb(a);
  double* M = smem;
  double* X = smem + 64 * DS;
  double* dsh = smem + 2 * 64 * DS;
  T* Tb = reinterpret_cast<T*>(smem + 2 * 64 * DS + 64);  // 64 x DS
  T* rdb = Tb + 64 * DS;                                  // 64: 1 / d of Tb's block
  if (a.Wprev) chain_block00<T, 8>(a, M, X);
  const bool chain_group = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8) == 0;  // (a uniform branch)
  for (int j = 0; j < nb; ++j) {
    const int tid = launder((int)threadIdx.x), lane = tid & 63;
    const int j0 = k0 + 64 * j, bj = panel_bsz(a, j);
    const bool more = j + 1 < nb;
    const int c = j + 1, r0 = k0 + 64 * c, rows = more ? panel_bsz(a, c) : 0;
    T* Lb = a.Lb0 + (int64_t)j * 64 * 64;
    if (chain_group) {
      CSTAMP(j0 / 64, 0);
      if (j == 0 && !a.Wprev)
        diag64_body<true, false, T, false, 4, NoHook, true, NoHook, 1, true>(K, ld, j0, bj, a.D, Lb, a.info, M, X, dsh,
                                                                             nullptr, NoHook(), nullptr, tid);
      else
        diag64_body<true, false, T, true, 4, NoHook, true, NoHook, 1, true>(K, ld, j0, bj, a.D, Lb, a.info, M, X, dsh,
                                                                            nullptr, NoHook(), nullptr, tid);
      CSTAMP(j0 / 64, 2);
      if (!more) break;
      __syncthreads();  // T1: the write-back's reads of M done
      CSTAMP(j0 / 64, 3);
      __syncthreads();  // T2: M holds the next diagonal block
      CSTAMP(j0 / 64, 5);
      continue;
    }
    // ======== bulk group
    const TMap<4> m(tid);
    const int arow = 16 * m.wr + (lane & 15);
    auto bar = [&]() { __syncthreads(); };
    bar();  // #1
    // I2: the previous transition's stores complete (DIAG / REG below)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();  // #2 (the chain group drained its write-back before it: DRAIN0)
    if (j >= 1 && tid == 256) {
      if (!(a.inject && j == 1)) st_sc1(&area[OP_DIAG + j - 1], 1u);
      st_sc1(&area[OP_REG + (j - 1) * OP_NBMAX + j], 1u);
    }
    if (!more) {  // the panel's last block: no block row below it
      for (int b = 3; b <= 10; ++b) bar();
      break;
    }
    bar();  // #3
    bar();  // #4
    bar();  // #5
    // I6: the next block row's operands (helper c stored them write-through)
    if (lane == 0) {  // every bulk wave polls for itself (no group barrier needed)
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (ld_sc1(&area[OP_READY + c]) == 0u) {
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS || ld_sc1(a.err) != 0u) {
          st_sc1(a.err, 1u);  // (the window runs on with stale data; the host reports the error)
          break;
        }
      }
    }
    CSTAMP_T(256, j0 / 64, 1);
    T aop[16];  // TRSM A operand: A(c, j)[arow][4 s + (lane >> 4)]
    {
      const T* Ar = K + (int64_t)(r0 + (arow < rows ? arow : 0)) * ld + j0 + (lane >> 4);
#pragma unroll
      for (int s = 0; s < 16; ++s) aop[s] = arow < rows ? ld_sc1(Ar + 4 * s) : T(0);
    }
    Acc<T> own[4];
    load_acc<T, true, true, 4>(m, own, K + (int64_t)r0 * ld + r0, ld, rows, rows);
    bar();  // #6
    bar();  // #7
    // TRSM column block n: tacc = A(c, j) X_n^T (mma_tile_lower's sequence for
    // acc[n]); T and 1 / d into LDS (L = T / d is formed where it is read)
    auto trsm_col = [&](auto nc) {
      constexpr int n = decltype(nc)::value;
      Acc<T> tacc = {T(0), T(0), T(0), T(0)};
      const int r = 16 * n + (lane & 15);
#pragma unroll
      for (int s = 0; s < 4 * (n + 1); ++s) {
        const int k = 4 * s + (lane >> 4);
        tacc = MF::mma(aop[s], k <= r ? (T)X[r * DS + k] : T(0), tacc);
        __builtin_amdgcn_sched_barrier(0);  // (no LDS reads hoisted: registers)
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) Tb[(16 * m.wr + MF::row(lane, g)) * DS + 16 * n + (lane & 15)] = tacc[g];
      if (m.wr == 0 && lane < 16) rdb[16 * n + lane] = T(1) / (T)dsh[16 * n + lane];
    };
    // own update with k block kb: own -= L[:, kb] W[:, kb]^T (mma_tile's s = 4 kb .. 4 kb + 3)
    auto own_kb = [&](int kb) {
#pragma unroll
      for (int s = 4 * kb; s < 4 * kb + 4; ++s) {
        const int k = 4 * s + (lane >> 4);
        const T av = -(Tb[arow * DS + k] * rdb[k]);
#pragma unroll
        for (int n = 0; n < 4; ++n) own[n] = MF::mma(av, Tb[(16 * n + (lane & 15)) * DS + k], own[n]);
        __builtin_amdgcn_sched_barrier(0);  // (no LDS reads hoisted: registers)
      }
    };
    // I8 (column pass 3): X_0, X_1 and D_0, D_1 final
    trsm_col(std::integral_constant<int, 0>{});
    trsm_col(std::integral_constant<int, 1>{});
    bar();  // #8
    // I9: X_2, D_2 final; Tb columns 0, 1 complete
    own_kb(0);
    own_kb(1);
    trsm_col(std::integral_constant<int, 2>{});
    bar();  // #9
    own_kb(2);  // I10
    bar();  // #10
    // transition: X_3 final (D_3 since #8)
    trsm_col(std::integral_constant<int, 3>{});
    bar();  // T1
    own_kb(3);
    // L(c, j) and W(c, j) from Tb (published after #2 of the next window): a
    // row's columns contiguous per wave-instruction
    {
      const int tb = tid - 256, cc = tb & 63;
      T* Lr = K + (int64_t)r0 * ld + j0;
      T* Wr = a.Wp + (int64_t)r0 * ldw + 64 * j;
      const T rdc = rdb[cc];
#pragma unroll 4
      for (int q = 0; q < 16; ++q) {
        const int rr = (tb >> 6) + 4 * q;
        if (rr < rows) {
          const T tv = Tb[rr * DS + cc];
          Lr[(int64_t)rr * ld + cc] = tv * rdc;
          st_sc1(&Wr[(int64_t)rr * ldw + cc], tv);
        }
      }
    }
    // the next diagonal block, straight into diag64_body's image
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = 16 * n + (lane & 15);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int row = 16 * m.wr + MF::row(lane, g);
        M[row * DS + col] = (row < rows && col <= row) ? (double)own[n][g] : (row == col ? 1.0 : 0.0);
      }
    }
    bar();  // T2
  }
  // the last block's DIAG (the chain group drains its write-back)
  if (chain_group) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && !(a.inject && nb == 1)) st_sc1(&area[OP_DIAG + nb - 1], 1u);
}

// ---- TILE WORKER: region block (c, q), 1 <= c < nb, q <= c: the look-ahead
// update with the previous panel, stored write-through, then TILE[c][q]
template <typename T, int NW>
__device__ __forceinline__ void tile_worker(const PanelArgs<T>& a, int t, double* smem) {
  const int tid = launder((int)threadIdx.x);
  const TMap<NW> m(tid);
  const int nb = panel_nb(a);
  int w = t - nb, c = 1;
  while (w > c) {
    w -= c + 1;
    ++c;
  }
  const int q = w, r0 = a.k0 + 64 * c, q0 = a.k0 + 64 * q, rows = panel_bsz(a, c), qrows = panel_bsz(a, q);
  Acc<T> upd[TMap<NW>::NN], tile[TMap<NW>::NN];
  zero_acc<T, TMap<NW>::NN>(upd);
  prev_update<T, NW>(tid, upd, a.Wprev + (int64_t)r0 * a.ldw, a.ldw, a.K + (int64_t)q0 * a.ld + a.kprev, a.ld, rows,
                     qrows, a.boprev, reinterpret_cast<T*>(smem), reinterpret_cast<T*>(smem + 64 * DS));
  T* dst = a.K + (int64_t)r0 * a.ld + q0;
  if (q == c) load_acc<T, false, true, NW>(m, tile, dst, a.ld, rows, rows);
  else load_acc<T, false, false, NW>(m, tile, dst, a.ld, rows, qrows);
#pragma unroll
  for (int i = 0; i < TMap<NW>::NN; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) tile[i][g] = tile[i][g] - upd[i][g];
  if (q == c) store_acc<T, true, true, NW>(m, tile, dst, a.ld, rows, rows);
  else store_acc<T, true, false, NW>(m, tile, dst, a.ld, rows, qrows);
  publish(&a.area[OP_TILE + c * OP_NBMAX + q]);
}

// ---- HELPER c: the TRSMs of its blocks j <= c - 2 and their strip updates,
// then READY[c]
template <typename T, int NW>
__device__ __forceinline__ void helper(const PanelArgs<T>& a, int c, double* smem, unsigned* sh_ok) {
  constexpr int NN = TMap<NW>::NN;
  T* const K = a.K;
  const int64_t ld = a.ld;
  const int k0 = a.k0, ldw = a.ldw;
  unsigned* const area = a.area;
  const int r0 = k0 + 64 * c, rows = panel_bsz(a, c);
  T* As = reinterpret_cast<T*>(smem);            // L(c, j) rows
  T* Bs = reinterpret_cast<T*>(smem + 64 * DS);  // L_jj^{-1}, then W pieces
  if (a.Wprev) {  // this row of region blocks, updated with the previous panel by the tile workers
    for (int q = 0; q <= c; ++q)
      if (!wait_flag(&area[OP_TILE + c * OP_NBMAX + q], a.err, sh_ok)) return;
  }
  for (int j = 0; j + 2 <= c; ++j) {
    const int tid = launder((int)threadIdx.x), lane = tid & 63;
    const TMap<NW> m(tid);
    const int j0 = k0 + 64 * j;
    T* Lb = a.Lb0 + (int64_t)j * 64 * 64;
    if (j || a.Wprev) stage_tile<T, true, NW>(tid, As, K + (int64_t)r0 * ld + j0, ld, rows, 64);
    else stage_tile<T, false, NW>(tid, As, K + (int64_t)r0 * ld + j0, ld, rows, 64);
    if (!wait_flag(&area[OP_DIAG + j], a.err, sh_ok)) return;
    stage_tile<T, true, NW>(tid, Bs, Lb, 64, 64, 64);
    T rd[NN];
#pragma unroll
    for (int i = 0; i < NN; ++i) rd[i] = T(1) / ld_sc1(&a.D[j0 + 16 * (m.n0 + i) + (lane & 15)]);
    __syncthreads();
    Acc<T> acc[NN];
    zero_acc<T, NN>(acc);
    mma_tile_lower<T, NW>(m, As, [&](int r, int k) { return Bs[r * DS + k]; }, acc);  // L_jj^{-1}: lower
    __syncthreads();
    Acc<T> lacc[NN];
#pragma unroll
    for (int i = 0; i < NN; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) lacc[i][g] = acc[i][g] * rd[i];
    store_acc<T, false, false, NW>(m, lacc, K + (int64_t)r0 * ld + j0, ld, rows, 64);
    store_acc<T, true, false, NW>(m, acc, a.Wp + (int64_t)r0 * ldw + 64 * j, ldw, rows, 64);
    publish(&area[OP_REG + j * OP_NBMAX + c]);
    put_acc<T, NW>(m, As, lacc);
    // strips: (c, q) -= L(c, j) W(q, j)^T, q = c, c-1 .. j+1: the own tile
    // (its W in registers) first, the tile whose W the chain publishes
    // (q = c-1 for j = c-2) last, its tile loaded before that wait -- so
    // READY[c] follows REG[c-2][c-1] by one strip
    for (int q = c; q > j; --q) {
      const int q0 = k0 + 64 * q, qrows = panel_bsz(a, q);
      Acc<T> tile[NN];
      if (q == c) load_acc<T, true, true, NW>(m, tile, K + (int64_t)r0 * ld + q0, ld, rows, rows);
      else load_acc<T, true, false, NW>(m, tile, K + (int64_t)r0 * ld + q0, ld, rows, qrows);
      if (q == c) {
        put_acc<T, NW>(m, Bs, acc);
      } else {
        if (!wait_flag(&area[OP_REG + j * OP_NBMAX + q], a.err, sh_ok)) return;
        stage_tile<T, true, NW>(tid, Bs, a.Wp + (int64_t)q0 * ldw + 64 * j, ldw, qrows, 64);
      }
      __syncthreads();
      mma_tile<T, true, NW>(m, As, [&](int r, int k) { return Bs[r * DS + k]; }, tile);
      if (q == c) store_acc<T, true, true, NW>(m, tile, K + (int64_t)r0 * ld + q0, ld, rows, rows);
      else store_acc<T, true, false, NW>(m, tile, K + (int64_t)r0 * ld + q0, ld, rows, qrows);
      __syncthreads();  // Bs reused by the next piece
    }
  }
  publish(&area[OP_READY + c]);
  HSTAMP(r0 / 64, 0);
}

// ---- the chain roles (tickets < nchain) in the NW-wave form
template <typename T, int NW>
__device__ __forceinline__ void chain_roles(const PanelArgs<T>& a, int t, double* smem, unsigned* sh_ok) {
  const int nb = panel_nb(a);
  if (t == 0) {
    if constexpr (NW == 8) chain8<T>(a, smem);
    else chain4<T>(a, smem, sh_ok);
  } else if (t >= nb) {
    tile_worker<T, NW>(a, t, smem);
  } else {
    helper<T, NW>(a, t, smem, sh_ok);
  }
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
  T* const K = a.K;
  const int64_t ld = a.ld;
  const int k0 = a.k0, N = a.N, ldw = a.ldw;
  const int ce = a.c1 < N ? a.c1 : N;
  const int nb = panel_nb(a);
  const int row0 = ce + 64 * r;
  const int rows = N - row0 < 64 ? N - row0 : 64;
  T* As = reinterpret_cast<T*>(smem);
  T* Bs = reinterpret_cast<T*>(smem + 64 * DS);
  T* Krow = K + (int64_t)row0 * ld;
  if (rows_prev) {
    for (int q = 0; q < nb; ++q) {
      const int tid = launder((int)threadIdx.x);
      const TMap<4> m(tid);
      const int q0 = k0 + 64 * q, qrows = panel_bsz(a, q);
      Acc<T> acc[4], tile[4];
      zero_acc<T, 4>(acc);
      prev_update<T, 4>(tid, acc, a.Wprev + (int64_t)row0 * ldw, ldw, K + (int64_t)q0 * ld + a.kprev, ld, rows, qrows,
                        a.boprev, As, Bs);
      load_acc<T, true, false, 4>(m, tile, Krow + q0, ld, rows, qrows);
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) tile[n][g] = tile[n][g] - acc[n][g];
      store_acc<T, false, false, 4>(m, tile, Krow + q0, ld, rows, qrows);
    }
  }
  // ---- TRSMs and strips of this chunk's rows.  Role 0 (the next panel's
  // first 64 rows) also accumulates that panel's block (0, 0) look-ahead
  // update W(rows, j) L(rows, j)^T over j -- exactly the chunks prev_update
  // would sum in the next chain role -- and leaves it in pre00_out.
  if (r == 0) HSTAMP(k0 / 64, 1);
  T* const p00 = r == 0 ? a.pre00_out : nullptr;
  Acc<T> a00[4];
  zero_acc<T, 4>(a00);
  bool ok = true;
  for (int j = 0; j < nb && ok; ++j) {
    const int tid = launder((int)threadIdx.x), lane = tid & 63;
    const TMap<4> m(tid);
    const int j0 = k0 + 64 * j, bj = panel_bsz(a, j);
    const T* Lb = a.Lb0 + (int64_t)j * 64 * 64;
    __syncthreads();  // previous block's strip finished reading As / Bs
    stage_tile<T, true, 4>(tid, As, Krow + j0, ld, rows, bj);
    if (!(ok = wait_flag(&a.area[OP_DIAG + j], a.err, sh_ok))) break;
    stage_tile<T, true, 4>(tid, Bs, Lb, 64, 64, 64);
    T rd[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = 16 * n + (lane & 15);
      rd[n] = col < bj ? T(1) / ld_sc1(&a.D[j0 + col]) : T(0);
    }
    __syncthreads();
    Acc<T> acc[4];
    zero_acc<T, 4>(acc);
    mma_tile_lower<T, 4>(m, As, [&](int rr, int k) { return Bs[rr * DS + k]; }, acc);  // L_jj^{-1}: lower
    __syncthreads();
    Acc<T> lacc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) lacc[n][g] = acc[n][g] * rd[n];
    store_acc<T, false, false, 4>(m, lacc, Krow + j0, ld, rows, bj);
    store_acc<T, false, false, 4>(m, acc, a.Wp + (int64_t)row0 * ldw + 64 * j, ldw, rows, bj);
    put_acc<T, 4>(m, As, lacc);
    if (p00) {  // a00 += W(rows, j) L(rows, j)^T (W staged in Bs, L in As)
      put_acc<T, 4>(m, Bs, acc);
      __syncthreads();
      mma_tile<T, false, 4>(m, Bs, [&](int rr, int k) { return As[rr * DS + k]; }, a00);
      __syncthreads();  // Bs is reused by the strips
    }
    // strips: (rows, q) -= L(rows, j) W(q, j)^T, q = j+1 .. nb-1
    for (int q = j + 1; q < nb; ++q) {
      const int q0 = k0 + 64 * q, qrows = panel_bsz(a, q);
      if (!(ok = wait_flag(&a.area[OP_REG + j * OP_NBMAX + q], a.err, sh_ok))) break;  // (its barrier also frees Bs)
      stage_tile<T, true, 4>(tid, Bs, a.Wp + (int64_t)q0 * ldw + 64 * j, ldw, qrows, bj);
      Acc<T> tile[4];
      load_acc<T, true, false, 4>(m, tile, Krow + q0, ld, rows, qrows);
      __syncthreads();
      mma_tile<T, true, 4>(m, As, [&](int rr, int k) { return Bs[rr * DS + k]; }, tile);
      store_acc<T, false, false, 4>(m, tile, Krow + q0, ld, rows, qrows);
      __syncthreads();
    }
  }
  if (p00 && ok) store_acc<T, false, false, 4>(TMap<4>(launder((int)threadIdx.x)), a00, p00, 64, 64, 64);
  if (r == 0) HSTAMP(k0 / 64, 2);
}

// draw a ticket: a chain role while any is left (when `chain_ok`), else a rows
// role (rows launch only); ~0u: none
template <typename T>
__device__ __forceinline__ unsigned draw_ticket(const PanelArgs<T>& a, bool chain_ok, bool rows_launch) {
  __shared__ unsigned sh_ticket;
  if (threadIdx.x == 0) {
    unsigned t = chain_ok ? atomicAdd(&a.area[OP_TICKET], 1u) : (unsigned)a.nchain;
    if (t >= (unsigned)a.nchain) t = rows_launch ? a.nchain + atomicAdd(&a.area[OP_TICKET + 1], 1u) : ~0u;
    sh_ticket = t;
  }
  __syncthreads();
  return sh_ticket;
}
}  // namespace

// The rows launch and, by default, the chain launch: 256 threads.
// amdgpu_waves_per_eu(2): <= 256 registers per lane (VGPR + AGPR), so a
// panel workgroup fits beside a trailing-GEMM workgroup (64 per lane at 4
// waves per SIMD) -- with more it waits for a CU with no GEMM at all.
template <typename T>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void panel_kernel(PanelArgs<T> a,
                                                                                           int rows_launch, int rows_prev) {
  // M, X: diag64_body's images (66.5 KB: a panel workgroup fits the LDS one
  // trailing-GEMM workgroup leaves free, so it is never starved of a CU)
  __shared__ __attribute__((aligned(16))) double smem[2 * 64 * DS + 64];
  __shared__ unsigned sh_ok;
  const unsigned tu = draw_ticket(a, true, rows_launch != 0);
  if (tu == ~0u) return;
  const int t = (int)tu;
  if (t == 0) HSTAMP(a.k0 / 64 + 1, 3);         // the chain role's workgroup starts
  if (t == a.nchain) HSTAMP(a.k0 / 64 + 2, 3);  // the first rows role starts
  if (t < a.nchain) {
    // s_setprio 3: the chain roles' waves win issue arbitration (matrix pipe
    // included) against the GEMM waves that share the CU
    __builtin_amdgcn_s_setprio(3);
    chain_roles<T, 4>(a, t, smem, &sh_ok);
  } else if (t < a.nchain + a.nrows) {
    rows_role<T>(a, t - a.nchain, rows_prev != 0, smem, &sh_ok);
  }
}

// The chain launch: 512 threads, the chain roles in their 8-wave form.  LDS
// 100 KB and <= 128 registers per lane (two waves per SIMD): the workgroup
// fits beside one trailing-GEMM workgroup (48 KB, 4 waves per SIMD at 64
// registers).  take = 0 (debug bit IPMZ_DEBUG_ROWS_CHAIN): no chain ticket is
// drawn, the rows launch runs every chain role in the 4-wave form.
template <typename T>
constexpr size_t chain_lds_bytes() {
  return (2 * 64 * DS + 64) * sizeof(double) + (64 * DS + 64) * sizeof(T);
}
// (dynamic LDS: with its static size the compiler would size the registers
// for the LDS-bound occupancy of 2 waves per SIMD, 256 each, and the
// workgroup would need a CU of its own)
template <typename T>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void panel_chain_kernel(PanelArgs<T> a,
                                                                                                 int take) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  __shared__ unsigned sh_ok;
  const unsigned tu = draw_ticket(a, take != 0, false);
  if (tu == ~0u) return;
  const int t = (int)tu;
  if (t == 0) HSTAMP(a.k0 / 64 + 1, 3);
  __builtin_amdgcn_s_setprio(3);
  chain_roles<T, 8>(a, t, smem, &sh_ok);
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
  const int dbg = debug_inject_mask();
  if (dbg & IPMZ_DEBUG_CHAIN8)  // the 512-thread chain launch, 8-wave chain roles
    hipLaunchKernelGGL(panel_chain_kernel<T>, dim3(a.nchain), dim3(512), chain_lds_bytes<T>(), st_chain, a,
                       (dbg & IPMZ_DEBUG_ROWS_CHAIN) ? 0 : 1);
  else if (dbg & IPMZ_DEBUG_ROWS_CHAIN)  // no chain ticket drawn: the rows launch runs every chain role
    hipLaunchKernelGGL(panel_chain_kernel<T>, dim3(a.nchain), dim3(512), chain_lds_bytes<T>(), st_chain, a, 0);
  else
    hipLaunchKernelGGL(panel_kernel<T>, dim3(a.nchain), dim3(256), 0, st_chain, a, 0, rows_prev ? 1 : 0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // the rows launch: every chain role and every rows role, should it run first
  // (with no rows below the region it is still launched when the chain launch
  // leaves the chain roles to it)
  if (a.nrows == 0 && !(dbg & IPMZ_DEBUG_ROWS_CHAIN)) return hipSuccess;
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
