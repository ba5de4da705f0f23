// The panel path of the blocked LDL^T: for one outer panel (columns
// [k0, c1), nb <= 8 inner blocks of 64), the column loop of
// LinearSolvers::ldlt_decomposition (LinearSolvers.cpp:20-40) restricted to
// those columns, as roles that hand off by flags.  Two launches of
// panel_kernel (256 threads) per panel -- the CHAIN launch (on the chain
// stream, padded with dynamic LDS to a CU per workgroup) and the ROWS launch
// (on the rows stream after the look-ahead strip update of the rows below) --
// and every workgroup takes its role from ticket counters (the chain roles'
// shared by both launches, so the panel completes in any dispatch order):
//
//   chain roles (the panel's diagonal region, first updated with the previous
//   panel; s_setprio 3):
//     ticket 0 = the CHAIN: for every inner block j, factor the 64 x 64
//       diagonal block (diag64_body), publish DIAG[j], the TRSM of the next
//       region block (j+1, j) and that block's own diagonal update; the
//       result IS the next diagonal block.  The whole critical path of the
//       panel lives on one CU (chain4: 4 waves, one step after the other;
//       an 8-wave form with the TRSM in the diagonal factor's shadow was
//       measured slower in round 5 -- 33 vs 19.5 us per block -- and removed).
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
//   strip tiles (rows launch, rows tickets before the rows roles, where the
//     host asks for them instead of the strip GEMM on the rows stream): tile
//     (r, q) of the rows below the region updated with the previous panel,
//     stored write-through; PREV[r] counts row r's tiles, and rows role r
//     waits for all nb of them.  Their inputs are complete when the launch
//     starts (stream order), so they wait for nothing and the rows roles
//     start as soon as their own row is updated, instead of behind a whole
//     strip GEMM launch.
//
// Every role computes each element with the same operations in the same order
// whichever launch holds it, so the factor is bitwise the same whichever
// launch holds a role (tests/test_gpu_panel_forms.py, debug bit
// IPMZ_DEBUG_ROWS_CHAIN: no chain launch, the rows launch takes every role).
//
// Flags: one area of IPMZ_PANEL_CTRL_WORDS words per outer panel (zeroed by
// one memset when the factorization starts); the sticky error word is shared.
// Hand-off protocol (cdna_hip_programming.md §6 Guideline 16, "Valid forms"
// row 1): data for another workgroup of a running launch is stored with sc1
// (relaxed agent-scope atomic stores), every storing wave drains vmcnt(0),
// a workgroup barrier, then one lane stores the flag; consumers poll with
// agent-scope loads and read the data with sc1 loads.
#include <atomic>

#include "common.h"
#include "diag64.h"
#include "kernels.h"
#include "sync.h"

namespace ipmz {

// -DIPMZ_CHAIN_STAMPS (tools/kbench "chainclk" only): s_memrealtime stamps of
// the chain role per 64-column block (k0 / 64 + j): 0 diag start, 1 READY[c]
// seen, 2 diag done, 3 operands loaded, 4 TRSM done, 5 next diagonal block
// formed; rows role 0: 6 DIAG seen, 7 TRSM (+ block (0, 0) sum) done, 8 strips
// done; helpers:
// READY[c] published; rows role 0: start, end; launches: first workgroup
// start per launch.
__device__ unsigned long long g_cstamp[IPMZ_CHAIN_STAMP_BLOCKS][16];
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
// the chain's column pass (diag64.h): 4 = colpass16_short<1>, the shorter
// per-pivot chain (in-panel block 20.0 -> 19.5-19.7 us, kbench chainclk
// N = 2560, profiles/r06_s/chain_cpv_ab.txt); 1 = colpass16_spec
#ifndef IPMZ_DIAG_CPV
#define IPMZ_DIAG_CPV 4
#endif
hipError_t chain_stamps(unsigned long long* c, unsigned long long* h) {  // DEBUG
  hipError_t e = hipMemcpyFromSymbol(c, HIP_SYMBOL(g_cstamp), sizeof(g_cstamp));
  if (e != hipSuccess) return e;
  return hipMemcpyFromSymbol(h, HIP_SYMBOL(g_hstamp), sizeof(g_hstamp));
}

namespace {
// ctrl words of a panel: OP_TICKET (chain tickets 0.., then rows tickets at
// OP_TICKET + 1), DIAG[j], REG[j][q], READY[c], TILE[c][q], RDONE[r]
enum { OP_TICKET = 0, OP_NRDY = 2, OP_R0 = 3, OP_DIAG = 4, OP_REG = 16, OP_READY = 96, OP_TILE = 128, OP_RDONE = 192, OP_PREV = 256 };
constexpr int OP_NBMAX = IPMZ_NBO_MAX / 64;
constexpr int OP_PREVMAX = IPMZ_PANEL_CTRL_WORDS - OP_PREV;  // rows roles that strip tiles can serve
static_assert(OP_DIAG + OP_NBMAX <= OP_REG && OP_REG + OP_NBMAX * OP_NBMAX <= OP_READY, "ctrl layout");
static_assert(OP_READY + OP_NBMAX <= OP_TILE, "ctrl layout");
static_assert(OP_TILE + OP_NBMAX * OP_NBMAX <= OP_RDONE, "ctrl layout");
static_assert(OP_RDONE + OP_NBMAX <= OP_PREV && OP_PREVMAX >= IPMZ_EARLY_CHAIN_MAX_N / 64, "panel ctrl area too small");

template <typename T>
using Acc = typename Mfma<T>::acc_t;

// The lane's place in a 64 x 64 tile in MFMA accumulator layout spread over
// NW waves: rows 16 wr + row(lane, g), column blocks n0 .. n0 + NN - 1
// (columns 16 n + (lane & 15)).  NW = 4: wave w holds row block w, every
// column block;
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
// ascale (optional, LDS): A's element (r, k) is As[r][k] * ascale[k] (one
// rounding: the L = W / d tile read from the W tile)
template <typename T, bool NEG, int NW, typename BF>
__device__ __forceinline__ void mma_tile(const TMap<NW>& m, const T* As, BF bf, Acc<T> (&acc)[TMap<NW>::NN],
                                         const T* ascale = nullptr) {
  typedef Mfma<T> MF;
  const int arow = 16 * m.wr + (m.lane & 15);
#pragma unroll 4
  for (int s = 0; s < 16; ++s) {
    const int k = 4 * s + (m.lane >> 4);
    const T av = ascale ? As[arow * DS + k] * ascale[k] : As[arow * DS + k];
    const T a = NEG ? -av : av;
#pragma unroll
    for (int i = 0; i < TMap<NW>::NN; ++i) acc[i] = MF::mma(a, bf(16 * (m.n0 + i) + (m.lane & 15), k), acc[i]);
  }
}

// One column block n of mma_tile: the same MFMAs into acc in the same order
// (so a tile computed this way is bitwise mma_tile's)
// (row block wr: the caller's, default the wave's)
template <typename T, bool NEG, int NW, typename BF>
__device__ __forceinline__ void mma_nblk(const TMap<NW>& m, const T* As, BF bf, Acc<T>& acc, int n,
                                         const T* ascale, int wr = -1) {
  typedef Mfma<T> MF;
  const int arow = 16 * (wr < 0 ? m.wr : wr) + (m.lane & 15);
#pragma unroll 4
  for (int s = 0; s < 16; ++s) {
    const int k = 4 * s + (m.lane >> 4);
    const T av = ascale ? As[arow * DS + k] * ascale[k] : As[arow * DS + k];
    const T a = NEG ? -av : av;
    acc = MF::mma(a, bf(16 * n + (m.lane & 15), k), acc);
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
template <typename T, int NW, bool SC = false>
__device__ __forceinline__ void prev_update(int tid, Acc<T> (&acc)[TMap<NW>::NN], const T* Wr, int64_t ldw,
                                            const T* Lr, int64_t ld, int rows, int qrows, int bop, T* As, T* Bs) {
  const TMap<NW> m(tid);
  T va[64 / NW], vb[64 / NW];
  fetch_tile<T, SC, NW>(tid, va, Wr, ldw, rows, bop < 64 ? bop : 64);
  fetch_tile<T, SC, NW>(tid, vb, Lr, ld, qrows, bop < 64 ? bop : 64);
  for (int kk = 0; kk < bop; kk += 64) {
    const int kw = bop - kk < 64 ? bop - kk : 64;
    __syncthreads();  // previous chunk's reads of As / Bs done
    put_tile<T, NW>(tid, As, va, rows, kw);
    put_tile<T, NW>(tid, Bs, vb, qrows, kw);
    __syncthreads();
    if (kk + 64 < bop) {
      const int kn = bop - kk - 64 < 64 ? bop - kk - 64 : 64;
      fetch_tile<T, SC, NW>(tid, va, Wr + kk + 64, ldw, rows, kn);
      fetch_tile<T, SC, NW>(tid, vb, Lr + kk + 64, ld, qrows, kn);
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
  int giveback;  // IPMZ_DEBUG_GIVEBACK: an early chain launch never sees RDONE (tests its 1 ms give-back)
  const T* Wprev;  // previous panel's W (nullptr: no look-ahead update in this launch pair)
  int kprev, boprev;
  const T* pre00_in;  // this panel's block (0, 0) update, accumulated by the previous rows role 0
  T* pre00_out;       // the next panel's, accumulated by rows role 0
  // the previous panel's ctrl area when its rows launch may still run beside
  // this launch: its rows roles r < OP_NBMAX (this panel's rows) raise
  // RDONE[r] once their L / W rows (and pre00) are stored write-through
  const unsigned* parea;
  int nchain;         // chain-role tickets
  int nrows;          // rows-role tickets
  int nprev;          // strip-tile tickets (nrows * nb or 0), before the rows roles
  int pre00w;         // 1: a PRE00 worker ticket after the rows roles sums pre00_out (else rows role 0)
  int wait_ready;     // 1 (chain launch): area[OP_NRDY] (panel_ready) within 1 ms, then acquire, before drawing a role
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
__device__ __forceinline__ bool chain_block00(const PanelArgs<T>& a, double* M, double* X) {
  __shared__ unsigned sh_w;
  if (a.parea && !wait_flag(const_cast<unsigned*>(&a.parea[OP_RDONE]), a.err, &sh_w)) return false;
  const int tid = launder((int)threadIdx.x);
  const TMap<NW> m(tid);
  const int k0 = a.k0, b0 = panel_bsz(a, 0);
  Acc<T> own[TMap<NW>::NN];
  if (a.pre00_in) {
    // accumulated by the previous panel's rows role 0 (the same MFMA order as
    // prev_update), so this role starts with the diagonal factor
    if (a.parea) load_acc<T, true, false, NW>(m, own, a.pre00_in, 64, 64, 64);
    else load_acc<T, false, false, NW>(m, own, a.pre00_in, 64, 64, 64);
  } else {
    zero_acc<T, TMap<NW>::NN>(own);
    const T* Wr = a.Wprev + (int64_t)k0 * a.ldw;
    const T* Lr = a.K + (int64_t)k0 * a.ld + a.kprev;
    if (a.parea)
      prev_update<T, NW, true>(tid, own, Wr, a.ldw, Lr, a.ld, b0, b0, a.boprev, reinterpret_cast<T*>(M),
                               reinterpret_cast<T*>(X));
    else
      prev_update<T, NW>(tid, own, Wr, a.ldw, Lr, a.ld, b0, b0, a.boprev, reinterpret_cast<T*>(M),
                         reinterpret_cast<T*>(X));
  }
  Acc<T> a0[TMap<NW>::NN];
  load_acc<T, false, true, NW>(m, a0, a.K + (int64_t)k0 * a.ld + k0, a.ld, b0, b0);
  put_diag_image<T, NW>(m, M, a0, own, b0);
  // (diag64_body's first barrier orders these stores before its reads)
  return true;
}

// ---- CHAIN, 4 waves (a 256-thread workgroup of either launch).  Per block
// j: the diagonal factor (diag64_body) with its write-back, then the TRSM of
// block (c, j), c = j + 1, and the own update of (c, c), which is the next
// diagonal block.  The operands of block row c are loaded before the
// write-back (their latency overlaps it; loaded unmasked -- a select would
// wait for the load -- the elements of rows past the matrix and above the
// diagonal only reach outputs that are never stored or used); the own update
// reads L = W / d from the W tile in LDS.
template <typename T>
__device__ __forceinline__ void chain4(const PanelArgs<T>& a, double* smem, unsigned* sh_ok) {
  typedef Mfma<T> MF;
  T* const K = a.K;
  const int64_t ld = a.ld;
  const int k0 = a.k0, ldw = a.ldw;
  unsigned* const area = a.area;
  const int nb = panel_nb(a);
  double* M = smem;
  double* X = smem + 64 * DS;
  double* dsh = smem + 2 * 64 * DS;         // 64 doubles (diag64_body's pivots)
  T* rdv = reinterpret_cast<T*>(dsh + 64);  // 64: 1 / d of the block in dsh
  if (a.Wprev && !chain_block00<T, 4>(a, M, X)) return;
  for (int j = 0; j < nb; ++j) {
    const int tid = launder((int)threadIdx.x), lane = tid & 63;
    const TMap<4> m(tid);
    const int j0 = k0 + 64 * j, bj = panel_bsz(a, j);
    CSTAMP(j0 / 64, 0);
    T* Lb = a.Lb0 + (int64_t)j * 64 * 64;
    const bool more = j + 1 < nb;
    const int c = j + 1, r0 = k0 + 64 * c, rows = more ? panel_bsz(a, c) : 0;
    // block row c's operands (helper c stored them write-through), loaded
    // before the write-back: A(c, j) for the TRSM, the own block (c, c)
    bool ok = true;
    T va[16];
    Acc<T> own[4];
    auto pre_wb = [&]() __attribute__((always_inline)) {
      if (!more) return;
      ok = wait_flag(&area[OP_READY + c], a.err, sh_ok);  // (uniform)
      CSTAMP(j0 / 64, 1);
      if (!ok) return;
      fetch_tile<T, true, 4>(tid, va, K + (int64_t)r0 * ld + j0, ld, rows, 64);
      const T* src = K + (int64_t)r0 * ld + r0;
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = 16 * m.wr + MF::row(lane, g);
          own[n][g] = ld_sc1(&src[(int64_t)(row < rows ? row : 0) * ld + 16 * n + (lane & 15)]);
        }
    };
    // block j >= 1: the own update of its block with W(j, j-1) (in X) beyond
    // column block 0 -- tiles (w, n), 1 <= n <= w, of wave w's rows -- runs
    // on waves 1..3 while wave 0 factors column block 0 (diag64_body's IDLE0:
    // that pass reads column block 0 only; X is first written after its
    // barrier); every wave drains its L / W stores before that barrier
    // (DRAIN0) and REG[j-1][j] is raised after it (POST2)
    auto idle0 = [&]() __attribute__((always_inline)) {
      const T* Wx = reinterpret_cast<const T*>(X);
      // two tiles per wave: wave 1 (1,1) (3,3), wave 2 (2,1) (2,2), wave 3 (3,1) (3,2)
      static_for<2>([&](auto hc) {
        constexpr int h = decltype(hc)::value;
        const int i = m.wr == 1 ? (h ? 3 : 1) : m.wr;                       // (wave-uniform)
        const int n = m.wr == 1 ? (h ? 3 : 1) : (m.wr == 2 ? 1 + h : 1 + h);
        Acc<T> t;
#pragma unroll
        for (int g = 0; g < 4; ++g) t[g] = (T)M[(16 * i + MF::row(lane, g)) * DS + 16 * n + (lane & 15)];
        mma_nblk<T, true, 4>(m, Wx, [&](int r, int k) { return Wx[r * DS + k]; }, t, n, rdv, i);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = 16 * i + MF::row(lane, g), col = 16 * n + (lane & 15);
          M[row * DS + col] = (row < bj && col <= row) ? (double)t[g] : (row == col ? 1.0 : 0.0);
        }
      });
    };
    auto post2 = [&]() __attribute__((always_inline)) {
      if (threadIdx.x == 0) st_sc1(&area[OP_REG + (j - 1) * OP_NBMAX + j], 1u);
    };
    if (j == 0 && !a.Wprev)
      diag64_body<true, false, T, false, 4, decltype(pre_wb), true, NoHook, IPMZ_DIAG_CPV, false, true, NoHook>(
          K, ld, j0, bj, a.D, Lb, a.info, M, X, dsh, nullptr, pre_wb, nullptr, tid);
    else if (j == 0)
      diag64_body<true, false, T, true, 4, decltype(pre_wb), true, NoHook, IPMZ_DIAG_CPV, false, true, NoHook>(
          K, ld, j0, bj, a.D, Lb, a.info, M, X, dsh, nullptr, pre_wb, nullptr, tid);
    else
      diag64_body<true, false, T, true, 4, decltype(pre_wb), true, decltype(idle0), IPMZ_DIAG_CPV, true, true, decltype(post2)>(
          K, ld, j0, bj, a.D, Lb, a.info, M, X, dsh, nullptr, pre_wb, nullptr, tid, idle0, nullptr, post2);
    CSTAMP(j0 / 64, 2);
    if (!more) {
      if (!(a.inject && j == 0)) publish(&area[OP_DIAG + j]);
      break;
    }
    if (!ok) return;
    // A(c, j) into M (free: the write-back has read L_jj), 1 / d of block j
    put_tile<T, 4>(tid, reinterpret_cast<T*>(M), va, rows, 64);
    if (tid < 64) rdv[tid] = T(1) / (T)dsh[tid];
    T rd[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) rd[n] = T(1) / (T)dsh[16 * n + (lane & 15)];
    // DIAG[j] (its write-back drained beside the operand loads; inject:
    // timeout tests only); publish's barrier also orders M and rdv
    if (!(a.inject && j == 0)) publish(&area[OP_DIAG + j]);
    else __syncthreads();
    CSTAMP(j0 / 64, 3);
    // TRSM: T = A(c, j) X_jj^T with X lower triangular (its upper part in
    // LDS is not meaningful: masked)
    Acc<T> acc[4];
    zero_acc<T, 4>(acc);
    mma_tile_lower<T, 4>(m, reinterpret_cast<const T*>(M),
                         [&](int r, int k) { return k <= r ? (T)X[r * DS + k] : T(0); }, acc);
    // the own block's loads are waited for here, before the L / W stores
    // (a wait at its first use after them would wait for those stores too)
#pragma unroll
    for (int n = 0; n < 4; ++n) asm volatile("" ::"v"(own[n]));
    __syncthreads();  // M reads done
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
    // own update (c, c) -= L(c, j) W(c, j)^T, column block 0 here (what
    // diag(c)'s first column pass reads), the rest in diag(c)'s IDLE0: W into
    // X (free: the TRSM's reads of X_jj are done), L = W / d read from it
    T* Wx = reinterpret_cast<T*>(X);
    put_acc<T, 4>(m, Wx, acc);
    __syncthreads();
    mma_nblk<T, true, 4>(m, Wx, [&](int r, int k) { return Wx[r * DS + k]; }, own[0], 0, rdv);
    CSTAMP(j0 / 64, 5);
    // the next diagonal block, straight into diag64_body's image (column
    // blocks >= 1 not yet updated: IDLE0 above, in the next iteration)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = 16 * n + (lane & 15);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int row = 16 * m.wr + MF::row(lane, g);
        M[row * DS + col] = (row < rows && col <= row) ? (double)own[n][g] : (row == col ? 1.0 : 0.0);
      }
    }
    // (diag64_body's first barrier orders these stores before its reads)
  }
}

// ---- TILE WORKER: region block (c, q), 1 <= c < nb, q <= c: the look-ahead
// update with the previous panel, stored write-through, then TILE[c][q]
template <typename T, int NW>
__device__ __forceinline__ void tile_worker(const PanelArgs<T>& a, int t, double* smem, unsigned* sh_ok) {
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
  const T* Wr = a.Wprev + (int64_t)r0 * a.ldw;
  const T* Lr = a.K + (int64_t)q0 * a.ld + a.kprev;
  T* As = reinterpret_cast<T*>(smem);
  T* Bs = reinterpret_cast<T*>(smem + 64 * DS);
  if (a.parea) {  // W rows c and L rows q from the previous panel's rows roles c and q
    if (!wait_flag(const_cast<unsigned*>(&a.parea[OP_RDONE + c]), a.err, sh_ok) ||
        !wait_flag(const_cast<unsigned*>(&a.parea[OP_RDONE + q]), a.err, sh_ok))
      return;
    prev_update<T, NW, true>(tid, upd, Wr, a.ldw, Lr, a.ld, rows, qrows, a.boprev, As, Bs);
  } else {
    prev_update<T, NW>(tid, upd, Wr, a.ldw, Lr, a.ld, rows, qrows, a.boprev, As, Bs);
  }
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

// ---- HELPER c: the TRSMs of its blocks j <= c - 2 and their strip
// updates, then READY[c]
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
  // The own tile (c, c) stays in registers over the steps, and tile (c, j+1),
  // final after step j's last strip, is carried in registers into step j+1
  // as its L(c, j+1) operand; the other tiles of the row go through global
  // with the next one's loads in flight during the current strip.
  const int jlast = c - 2;
  Acc<T> own[NN], carry[NN];
  if (jlast >= 0) {
    const TMap<NW> m(launder((int)threadIdx.x));
    if (a.Wprev) load_acc<T, true, true, NW>(m, own, K + (int64_t)r0 * ld + r0, ld, rows, rows);
    else load_acc<T, false, true, NW>(m, own, K + (int64_t)r0 * ld + r0, ld, rows, rows);
  }
  for (int j = 0; j <= jlast; ++j) {
    const int tid = launder((int)threadIdx.x), lane = tid & 63;
    const TMap<NW> m(tid);
    const int j0 = k0 + 64 * j;
    T* Lb = a.Lb0 + (int64_t)j * 64 * 64;
    if (j == 0) {
      if (a.Wprev) stage_tile<T, true, NW>(tid, As, K + (int64_t)r0 * ld + j0, ld, rows, 64);
      else stage_tile<T, false, NW>(tid, As, K + (int64_t)r0 * ld + j0, ld, rows, 64);
    } else {
      put_acc<T, NW>(m, As, carry);
    }
    Acc<T> tA[NN];  // tile (c, c-1): the first strip's, loaded before the DIAG wait
    load_acc<T, true, false, NW>(m, tA, K + (int64_t)r0 * ld + k0 + 64 * (c - 1), ld, rows, panel_bsz(a, c - 1));
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
    put_acc<T, NW>(m, Bs, acc);
    __syncthreads();
    mma_tile<T, true, NW>(m, As, [&](int r, int k) { return Bs[r * DS + k]; }, own);  // (c, c) -= L W^T
    __syncthreads();
    // strips q = c-1 .. j+1: the tile whose W the chain publishes (q = j+1)
    // last, so READY[c] follows that REG flag by one strip
    for (int q = c - 1; q > j; --q) {
      const int q0 = k0 + 64 * q, qrows = panel_bsz(a, q);
      if (!wait_flag(&area[OP_REG + j * OP_NBMAX + q], a.err, sh_ok)) return;
      T vw[64 / NW];
      fetch_tile<T, true, NW>(tid, vw, a.Wp + (int64_t)q0 * ldw + 64 * j, ldw, qrows, 64);
      Acc<T> tB[NN];
      if (q - 1 > j)
        load_acc<T, true, false, NW>(m, tB, K + (int64_t)r0 * ld + q0 - 64, ld, rows, panel_bsz(a, q - 1));
      put_tile<T, NW>(tid, Bs, vw, qrows, 64);
      __syncthreads();
      mma_tile<T, true, NW>(m, As, [&](int r, int k) { return Bs[r * DS + k]; }, tA);
      if (q == j + 1 && j < jlast) {
#pragma unroll
        for (int i = 0; i < NN; ++i)
#pragma unroll
          for (int g = 0; g < 4; ++g) carry[i][g] = tA[i][g];
      } else {
        store_acc<T, true, false, NW>(m, tA, K + (int64_t)r0 * ld + q0, ld, rows, qrows);
      }
      __syncthreads();  // Bs reused by the next piece
#pragma unroll
      for (int i = 0; i < NN; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) tA[i][g] = tB[i][g];
    }
  }
  if (jlast >= 0) {
    const TMap<NW> m(launder((int)threadIdx.x));
    store_acc<T, true, true, NW>(m, own, K + (int64_t)r0 * ld + r0, ld, rows, rows);
  }
  publish(&area[OP_READY + c]);
  HSTAMP(r0 / 64, 0);
}

// ---- the chain roles (tickets < nchain) in the NW-wave form
template <typename T>
__device__ __forceinline__ void chain_roles(const PanelArgs<T>& a, int t, double* smem, unsigned* sh_ok) {
  const int nb = panel_nb(a);
  if (t == 0) chain4<T>(a, smem, sh_ok);
  else if (t >= nb) tile_worker<T, 4>(a, t, smem, sh_ok);
  else helper<T, 4>(a, t, smem, sh_ok);
}

// ---- a rows role (rows ticket r): the 64 rows from ce + 64 r.  Every
// operand another role of this panel produced is read with agent-scope loads
// (the producer may be in the other launch).  With strip tiles (a.nprev),
// it first waits for its row's look-ahead update with the previous panel.
template <typename T>
__device__ __forceinline__ void rows_role(const PanelArgs<T>& a, int r, double* smem, unsigned* sh_ok) {
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
  // this row's strip tiles (rows tickets drawn before this one: running or done)
  if (a.nprev && !wait_flag_ge(&a.area[OP_PREV + r], (unsigned)nb, a.err, sh_ok)) return;
  // ---- TRSMs and strips of this chunk's rows.  Role 0 (the next panel's
  // first 64 rows) also accumulates that panel's block (0, 0) look-ahead
  // update W(rows, j) L(rows, j)^T over j -- exactly the chunks prev_update
  // would sum in the next chain role -- and leaves it in pre00_out.
  if (r == 0) HSTAMP(k0 / 64, 1);
  T* const p00 = r == 0 && !a.pre00w ? a.pre00_out : nullptr;
  const bool r0w = r == 0 && a.pre00w;  // R0 counts this role's finished blocks for the PRE00 worker
  const bool wt = r < OP_NBMAX;  // rows of the next panel's diagonal region: RDONE[r]
  Acc<T> a00[4], carry[4];
  zero_acc<T, 4>(a00);
  __shared__ unsigned sh_pk;
  bool ok = true;
  for (int j = 0; j < nb && ok; ++j) {
    const int tid = launder((int)threadIdx.x), lane = tid & 63;
    const TMap<4> m(tid);
    const int j0 = k0 + 64 * j, bj = panel_bsz(a, j);
    __syncthreads();  // previous block's strip finished reading As / Bs
    if (j == 0) stage_tile<T, true, 4>(tid, As, Krow + j0, ld, rows, bj);
    else put_acc<T, 4>(m, As, carry);  // tile (rows, j), final after block j-1's first strip
    if (!(ok = wait_flag(&a.area[OP_DIAG + j], a.err, sh_ok))) break;
    if (r == 0) CSTAMP(j0 / 64, 6);
    stage_tile<T, true, 4>(tid, Bs, a.Lb0 + (int64_t)j * 64 * 64, 64, 64, 64);
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
    // (R0: block j-1's L / W stores, long issued, drained here, off the MFMAs' way)
    if (r0w && j > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (r0w && j > 0 && threadIdx.x == 0)
      __hip_atomic_store(&a.area[OP_R0], (unsigned)j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    Acc<T> lacc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g) lacc[n][g] = acc[n][g] * rd[n];
    if (wt) {  // the next panel's launch may read them before this launch ends
      store_acc<T, true, false, 4>(m, lacc, Krow + j0, ld, rows, bj);
      store_acc<T, true, false, 4>(m, acc, a.Wp + (int64_t)row0 * ldw + 64 * j, ldw, rows, bj);
    } else {
      store_acc<T, false, false, 4>(m, lacc, Krow + j0, ld, rows, bj);
      store_acc<T, false, false, 4>(m, acc, a.Wp + (int64_t)row0 * ldw + 64 * j, ldw, rows, bj);
    }
    put_acc<T, 4>(m, As, lacc);
    if (p00) put_acc<T, 4>(m, Bs, acc);  // W, for a00 below
    if (r == 0) CSTAMP(j0 / 64, 7);
    // strips: (rows, q) -= L(rows, j) W(q, j)^T, q = nb-1 .. j+1.  Their REG
    // flags are polled together (the helpers raise them well ahead), the
    // next strip's W and A tiles load during this one's MFMAs, and tile
    // (rows, j+1), the next block's TRSM operand, the last one, stays in
    // registers (carry) instead of a store and a reload.  (The poll's barrier
    // frees Bs.)
    if (!(ok = wait_flags(&a.area[OP_REG + j * OP_NBMAX + j + 1], nb - j - 1, nullptr, a.err, sh_ok, &sh_pk)))
      break;
    if (j + 1 < nb) {
      T vw[16];
      Acc<T> nxt[4];
      auto fetch = [&](int q) {
        const int qrows = panel_bsz(a, q);
        fetch_tile<T, true, 4>(tid, vw, a.Wp + (int64_t)(k0 + 64 * q) * ldw + 64 * j, ldw, qrows, bj);
        load_acc<T, true, false, 4>(m, nxt, Krow + k0 + 64 * q, ld, rows, qrows);
      };
      fetch(nb - 1);
      if (p00) {  // a00 += W(rows, j) L(rows, j)^T (W in Bs, L in As), beside the first strip's loads
        mma_tile<T, false, 4>(m, Bs, [&](int rr, int k) { return As[rr * DS + k]; }, a00);
        __syncthreads();
      }
      for (int q = nb - 1; q > j; --q) {
        const int q0 = k0 + 64 * q, qrows = panel_bsz(a, q);
        put_tile<T, 4>(tid, Bs, vw, qrows, bj);
        Acc<T> tile[4];
#pragma unroll
        for (int n = 0; n < 4; ++n) tile[n] = nxt[n];
        __syncthreads();
        if (q - 1 > j) fetch(q - 1);
        mma_tile<T, true, 4>(m, As, [&](int rr, int k) { return Bs[rr * DS + k]; }, tile);
        if (q == j + 1) {
#pragma unroll
          for (int n = 0; n < 4; ++n) carry[n] = tile[n];
        } else {
          store_acc<T, false, false, 4>(m, tile, Krow + q0, ld, rows, qrows);
        }
        __syncthreads();  // Bs reads done
      }
    } else if (p00) {
      mma_tile<T, false, 4>(m, Bs, [&](int rr, int k) { return As[rr * DS + k]; }, a00);
    }
    if (r == 0) CSTAMP(j0 / 64, 8);
  }
  if (p00 && ok) store_acc<T, true, false, 4>(TMap<4>(launder((int)threadIdx.x)), a00, p00, 64, 64, 64);
  if (r0w && ok) {  // the PRE00 worker raises RDONE[0]
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(&a.area[OP_R0], (unsigned)nb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (wt && ok) {
    publish(&a.area[OP_RDONE + r]);
  }
  if (wt) HSTAMP(k0 / 64 + r, 2);
}

// ---- the PRE00 worker (the last rows ticket, strip-tile panels): the next
// panel's block (0, 0) look-ahead update W(rows 0, j) L(rows 0, j)^T summed
// over j as rows role 0 finishes each block (R0) -- the same MFMAs in the same
// order as role 0 sums it otherwise, off that role's path -- then pre00_out
// and RDONE[0] (role 0's rows are final too: R0 = nb).
template <typename T>
__device__ __forceinline__ void pre00_worker(const PanelArgs<T>& a, double* smem, unsigned* sh_ok) {
  const int nb = panel_nb(a);
  const int ce = a.c1 < a.N ? a.c1 : a.N;
  const int rows = a.N - ce < 64 ? a.N - ce : 64;
  T* As = reinterpret_cast<T*>(smem);
  T* Bs = reinterpret_cast<T*>(smem + 64 * DS);
  Acc<T> a00[4];
  zero_acc<T, 4>(a00);
  for (int j = 0; j < nb; ++j) {
    const int tid = launder((int)threadIdx.x);
    const TMap<4> m(tid);
    const int bj = panel_bsz(a, j);
    if (!wait_flag_ge(&a.area[OP_R0], (unsigned)(j + 1), a.err, sh_ok)) return;  // (its barrier frees As / Bs)
    stage_tile<T, true, 4>(tid, As, a.K + (int64_t)ce * a.ld + a.k0 + 64 * j, a.ld, rows, bj);  // L
    stage_tile<T, true, 4>(tid, Bs, a.Wp + (int64_t)ce * a.ldw + 64 * j, a.ldw, rows, bj);     // W
    __syncthreads();
    mma_tile<T, false, 4>(m, Bs, [&](int rr, int k) { return As[rr * DS + k]; }, a00);
  }
  store_acc<T, true, false, 4>(TMap<4>(launder((int)threadIdx.x)), a00, a.pre00_out, 64, 64, 64);
  publish(&a.area[OP_RDONE]);
}

// ---- a STRIP TILE (rows ticket u < nprev): tile (r, q), r = u / nb, of the
// rows below the region, A[rows r, block q] -= W_prev[rows r] L_prev[q]^T --
// the tile the strip GEMM on the rows stream computes otherwise, here in the
// rows launch so that rows role r starts once its own nb tiles are done (its
// inputs: the previous rows launch's W and L rows, complete in stream order).
// Stored write-through, then PREV[r] += 1.
template <typename T>
__device__ __forceinline__ void strip_tile(const PanelArgs<T>& a, int u, double* smem) {
  const int nb = panel_nb(a);
  const int r = u / nb, q = u - r * nb;
  const int ce = a.c1 < a.N ? a.c1 : a.N;
  const int row0 = ce + 64 * r, rows = a.N - row0 < 64 ? a.N - row0 : 64;
  const int q0 = a.k0 + 64 * q, qrows = panel_bsz(a, q);
  const int tid = launder((int)threadIdx.x);
  const TMap<4> m(tid);
  Acc<T> upd[4], tile[4];
  zero_acc<T, 4>(upd);
  prev_update<T, 4>(tid, upd, a.Wprev + (int64_t)row0 * a.ldw, a.ldw, a.K + (int64_t)q0 * a.ld + a.kprev, a.ld, rows,
                    qrows, a.boprev, reinterpret_cast<T*>(smem), reinterpret_cast<T*>(smem + 64 * DS));
  T* dst = a.K + (int64_t)row0 * a.ld + q0;
  load_acc<T, false, false, 4>(m, tile, dst, a.ld, rows, qrows);
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int g = 0; g < 4; ++g) tile[n][g] = tile[n][g] - upd[n][g];
  store_acc<T, true, false, 4>(m, tile, dst, a.ld, rows, qrows);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(&a.area[OP_PREV + r], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A chain launch started beside the previous panel's rows launch (a.parea):
// that launch's RDONE[0] (this panel's first block row, and its block (0, 0)
// update) -- and, with a.wait_ready, the panel's READY-TO-FACTOR word (the B
// stream's look-ahead update of its columns, panel_ready) -- within 1 ms,
// else no role is drawn: the launch may have been dispatched ahead of what
// it waits for (a serialized dispatch, rocprofv3 --pmc), and the rows launch
// of this panel, queued behind both on its stream, then takes every chain
// role.  Once RDONE[0] is up that rows launch is running, and the roles wait
// for its other rows with their own flags (RDONE[c] in the tile workers), so
// the chain starts its first block without waiting for the slowest of them.
// The ready word is followed by an agent-scope acquire (cdna_hip_programming.md
// §6 G16 consumer form: one relaxed poll, one acquire, then plain loads of
// the update's output).  true: draw.
template <typename T>
__device__ __forceinline__ bool prev_rows_ready(const PanelArgs<T>& a) {
  if (!a.parea && !a.wait_ready) return true;
  __shared__ unsigned sh_rr;
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool rows = !a.parea, ready = !a.wait_ready;
    unsigned ok = 0;
    for (;;) {
      if (!rows)
        rows = !a.giveback && __hip_atomic_load(&a.parea[OP_RDONE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
      if (!ready) ready = __hip_atomic_load(&a.area[OP_NRDY], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
      if (rows && ready) {
        ok = 1;
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > 100000ull) break;  // 1 ms
      __builtin_amdgcn_s_sleep(2);
    }
    if (ok && a.wait_ready) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    sh_rr = ok;
  }
  __syncthreads();
  return sh_rr != 0;
}

// draw a role: the CHAIN (ticket 0) if it is still unclaimed, else the next
// chain ticket while any is left, else -- rows launch -- a rows ticket.
// ~0u: none
template <typename T>
__device__ __forceinline__ unsigned draw_ticket(const PanelArgs<T>& a, bool rows_launch) {
  __shared__ unsigned sh_ticket;
  if (threadIdx.x == 0) {
    unsigned t = ~0u;
    const unsigned k = atomicAdd(&a.area[OP_TICKET], 1u);
    if (k < (unsigned)a.nchain) t = k;
    else if (rows_launch) t = a.nchain + atomicAdd(&a.area[OP_TICKET + 1], 1u);
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
                                                                                           int rows_launch) {
  // M, X: diag64_body's images (66.5 KB: a panel workgroup fits the LDS one
  // trailing-GEMM workgroup leaves free, so it is never starved of a CU)
  __shared__ __attribute__((aligned(16))) double smem[2 * 64 * DS + 64 + 64];
  __shared__ unsigned sh_ok;
  if (!rows_launch && blockIdx.x == 0) HSTAMP(a.k0 / 64 + 3, 3);  // the chain launch is dispatched
  if (!rows_launch && !prev_rows_ready(a)) return;
  const unsigned tu = draw_ticket(a, rows_launch != 0);
  if (tu == ~0u) return;
  const int t = (int)tu;
  if (t == 0) HSTAMP(a.k0 / 64 + 1, 3);         // the chain role's workgroup starts
  if (t == a.nchain) HSTAMP(a.k0 / 64 + 2, 3);  // the first rows role starts
  if (t < a.nchain) {
    // s_setprio 3: the chain roles' waves win issue arbitration (matrix pipe
    // included) against the GEMM waves that share the CU
    __builtin_amdgcn_s_setprio(3);
    chain_roles<T>(a, t, smem, &sh_ok);
  } else if (t < a.nchain + a.nprev + a.nrows) {
    if (t < a.nchain + a.nprev) strip_tile<T>(a, t - a.nchain, smem);
    else rows_role<T>(a, t - a.nchain - a.nprev, smem, &sh_ok);
  } else if (t < a.nchain + a.nprev + a.nrows + a.pre00w) {
    pre00_worker<T>(a, smem, &sh_ok);
  }
}

// ---------------------------------------------------------------------------
// dynamic LDS of the chain launch on top of panel_kernel's static 66.5 KB.
// 95 KB in all: more than a CU has left beside another panel workgroup
// (66.5 KB), so no two share a CU, while one trailing-GEMM workgroup (48 KB)
// still fits beside it.  113 KB where the order left from the panel is small
// (<= IPMZ_EARLY_CHAIN_MAX_N: the chain is the critical path): no GEMM
// workgroup beside it either
// (kbench N = 2560: 1.15 -> 1.10 ms; at N = 11264, where the trailing GEMM
// is, 10.97 -> 11.2 ms, so not there; profiles/r05_s/chain_lds_pad_ab.txt).
// 144 KB where the whole factor is that small (C2): not even a 64 x 64
// strip-GEMM workgroup (24 KB) beside it (C2 724 -> 734 steps/s; the same
// for C3's tail panels: 75.7 -> 74.6, so not there; profiles/r06_s8)
template <typename T>
static size_t chain_lds_pad(int Nleft, int N) {
  constexpr size_t own = (2 * 64 * DS + 64 + 64) * sizeof(double) + 64;
  constexpr size_t big = 113 * 1024, small = 95 * 1024, whole = 144 * 1024;
  // the attribute per device (a process may factor on several): 0 not yet
  // set, 1 set, 2 refused (then no padding)
  static std::atomic<unsigned char> state[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  unsigned char st = state[dev].load(std::memory_order_acquire);
  if (st == 0) {
    st = hipFuncSetAttribute(reinterpret_cast<const void*>(&panel_kernel<T>),
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)(whole - own)) == hipSuccess ? 1 : 2;
    state[dev].store(st, std::memory_order_release);
  }
  if (st != 1) return 0;
  if (N <= IPMZ_EARLY_CHAIN_MAX_N) return whole - own;
  return (Nleft <= IPMZ_EARLY_CHAIN_MAX_N ? big : small) - own;
}

template <typename T>
static hipError_t panel_launch_t(T* K, int64_t ld, int N, int k0, int bo, T* D, T* Lb0, T* Wp, int ldw,
                                 const T* pre00_in, T* pre00_out, int* info,
                                 unsigned* area, unsigned* err, const T* Wprev, int kprev, int boprev, bool rows_prev,
                                 hipStream_t st_chain, hipStream_t st_rows, const unsigned* parea,
                                 bool wait_ready) {
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
  a.parea = parea;
  a.giveback = (debug_inject_mask() & IPMZ_DEBUG_GIVEBACK) ? 1 : 0;
  // chain + nb - 1 helpers (+ one tile worker per region block below the
  // diagonal block (0, 0) when the look-ahead update is applied here)
  a.nchain = nb + (Wprev ? nb * (nb + 1) / 2 - 1 : 0);
  a.nrows = ce < N ? (N - ce + 63) / 64 : 0;
  // rows_prev: the look-ahead update of the rows below the region with the
  // previous panel as strip tiles of the rows launch (else the caller ran it)
  if (rows_prev && (!Wprev || a.nrows > OP_PREVMAX)) return hipErrorInvalidValue;
  a.nprev = rows_prev ? a.nrows * nb : 0;
  a.pre00w = (a.nprev && pre00_out) ? 1 : 0;
  a.wait_ready = wait_ready ? 1 : 0;
  const int dbg = debug_inject_mask();
  if (!(dbg & IPMZ_DEBUG_ROWS_CHAIN)) {
    // every chain role; the padding (dynamic LDS) makes each of its
    // workgroups hold a CU with no other panel workgroup (the chain's
    // barrier-bound blocks lose a third of their speed beside a helper)
    hipLaunchKernelGGL(panel_kernel<T>, dim3(a.nchain), dim3(256), chain_lds_pad<T>(N - k0, N), st_chain, a, 0);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // the rows launch: every chain role and every rows role, should it run first
  // (with no rows below the region it is still launched when the chain launch
  // may leave the chain roles to it: an early chain launch gives them back
  // after 1 ms without the previous rows launch's RDONE flags -- without
  // this launch the last panel would then never be factored, which
  // test_gpu_panel_forms.py's give-back form found in round 6)
  if (a.nrows == 0 && !parea && !(dbg & IPMZ_DEBUG_ROWS_CHAIN)) return hipSuccess;
  // (the rows launch is ordered after the B stream's update by its stream:
  // it never polls the ready flag -- spinning, its many workgroups could
  // hold the CUs that update needs)
  a.wait_ready = 0;
  hipLaunchKernelGGL(panel_kernel<T>, dim3(a.nchain + a.nprev + a.nrows + a.pre00w), dim3(256), 0, st_rows, a, 1);
  return hipGetLastError();
}
hipError_t panel_factor(double* K, int64_t ld, int N, int k0, int bo, double* D, double* Lb0, double* Wp, int ldw,
                        const double* pre00_in, double* pre00_out, int* info, unsigned* area, unsigned* err,
                        const double* Wprev, int kprev, int boprev, bool rows_prev, hipStream_t st_chain,
                        hipStream_t st_rows, const unsigned* parea, bool wait_ready) {
  return panel_launch_t<double>(K, ld, N, k0, bo, D, Lb0, Wp, ldw, pre00_in, pre00_out, info, area, err, Wprev, kprev,
                                boprev, rows_prev, st_chain, st_rows, parea, wait_ready);
}
hipError_t panel_factor(float* K, int64_t ld, int N, int k0, int bo, float* D, float* Lb0, float* Wp, int ldw,
                        const float* pre00_in, float* pre00_out, int* info, unsigned* area, unsigned* err,
                        const float* Wprev, int kprev, int boprev, bool rows_prev, hipStream_t st_chain,
                        hipStream_t st_rows, const unsigned* parea, bool wait_ready) {
  return panel_launch_t<float>(K, ld, N, k0, bo, D, Lb0, Wp, ldw, pre00_in, pre00_out, info, area, err, Wprev, kprev,
                               boprev, rows_prev, st_chain, st_rows, parea, wait_ready);
}

// READY-TO-FACTOR of a panel (its area's OP_NRDY word): one relaxed
// agent-scope store by a one-thread launch, ordered on its stream after the
// look-ahead update it stands for -- whose stores that launch's end released
// (debug bit IPMZ_DEBUG_READY_LATE: the word is raised 3 ms late, so every
// chain launch that waits for it gives its roles back to its rows launch --
// the path a serialized dispatch takes; tests/test_gpu_panel_forms.py)
__global__ void panel_ready_kernel(unsigned* w, unsigned long long delay) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < delay) __builtin_amdgcn_s_sleep(64);
  __hip_atomic_store(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
hipError_t panel_ready(unsigned* area, hipStream_t st) {
  const unsigned long long delay = (debug_inject_mask() & IPMZ_DEBUG_READY_LATE) ? 300000ull : 0ull;
  hipLaunchKernelGGL(panel_ready_kernel, dim3(1), dim3(1), 0, st, area + OP_NRDY, delay);
  return hipGetLastError();
}

}  // namespace ipmz
