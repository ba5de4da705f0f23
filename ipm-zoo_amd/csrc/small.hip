// Whole LDL^T of one small KKT matrix per workgroup (config C4: batches of
// N = 320 systems).  Replaces LinearSolvers::ldlt_decomposition
// (LinearSolvers.cpp:14-42) for the batched path: same factor (unit-lower L
// in the strict lower triangle of K, D, the 1e-8 zero-pivot rule inside
// diag64_body), blocked by 64 columns, right-looking, every step inside ONE
// workgroup -- no launch boundaries, no inter-workgroup hand-offs:
//   for each 64-column block J:
//     diag64_body: factor the diagonal block (L_JJ, D_J, L_JJ^{-1})
//     TRSM  : for every 64-row chunk c below: W_c = A[c, J] L_JJ^{-T},
//             L[c, J] = W_c / D_J                       (f64 MFMA 16x16x4)
//     update: A[c, q] -= L[c, J] W_q^T, J < q <= c      (f64 MFMA 16x16x4)
// The multi-launch batched factor paid a launch + a grid-wide drain per
// inner block and per update (and left half the chip idle at 128 QPs per
// GPU); here the only serialization is the algorithm's own.  LDS: the two
// 64 x DS operand tiles double as diag64_body's M and X (66.5 KB).  Eight
// waves (two per SIMD) split every 64 x 64 MFMA tile so one wave's LDS and
// memory waits overlap the other's MFMAs; operand tiles for the next step
// are loaded into registers while the current one computes.
#include <cstdio>
#include <type_traits>

#include "ipmz.h"
#include "common.h"
#include "kernels.h"
#include "diag64.h"
#include "sync.h"

namespace ipmz {

namespace {
typedef Mfma<double> MF;
typedef MF::acc_t acc_t;

// SNW waves per workgroup (8: two per SIMD)
template <int SNW>
struct Cfg {
  static constexpr int SNT = 64 * SNW;        // threads
  static constexpr int SFR = 64 / SNW;        // tile rows fetched per thread
  static constexpr int SNN = 4 * 4 / SNW;     // 16-column MFMA blocks per wave (rows: 16 (w & 3)..)
};

// 64 x 64 tile rows [0, nrows) of a row-major source (row stride lds): wave w
// loads rows w, w+SNW, ... (one 512-byte row per load instruction); rows
// past nrows read row 0 and are zeroed on the LDS store.
template <int SNW>
__device__ __forceinline__ void tile_fetch(const double* __restrict__ src, int64_t lds, int nrows,
                                           double (&v)[Cfg<SNW>::SFR], int tid = threadIdx.x) {
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int i = 0; i < Cfg<SNW>::SFR; ++i) {
    const int rr = wave + SNW * i;
    v[i] = src[(int64_t)(rr < nrows ? rr : 0) * lds + lane];
  }
}
// the same with agent-scope loads (data another workgroup of the launch wrote)
template <int SNW>
__device__ __forceinline__ void tile_fetch_sc(const double* __restrict__ src, int64_t lds, int nrows,
                                              double (&v)[Cfg<SNW>::SFR]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < Cfg<SNW>::SFR; ++i) {
    const int rr = wave + SNW * i;
    v[i] = ld_sc1(&src[(int64_t)(rr < nrows ? rr : 0) * lds + lane]);
  }
}
template <int SNW>
__device__ __forceinline__ void tile_put(double* dst, int nrows, const double (&v)[Cfg<SNW>::SFR],
                                         int tid = threadIdx.x) {
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int i = 0; i < Cfg<SNW>::SFR; ++i) {
    const int rr = wave + SNW * i;
    dst[rr * DS + lane] = rr < nrows ? v[i] : 0.0;
  }
}
// the same, column `lane` scaled by s (W = L D staged from an L tile)
template <int SNW>
__device__ __forceinline__ void tile_put_scaled(double* dst, int nrows, const double (&v)[Cfg<SNW>::SFR], double s,
                                                int tid) {
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int i = 0; i < Cfg<SNW>::SFR; ++i) {
    const int rr = wave + SNW * i;
    dst[rr * DS + lane] = rr < nrows ? v[i] * s : 0.0;
  }
}
// this wave's part of the 64 x 64 result: rows 16 (w & 3) .. +15, column
// blocks n0 + (0 .. SNN-1), n0 = SNN (w >> 2)
__device__ __forceinline__ int tile_r0(int tid = threadIdx.x) { return 16 * ((tid >> 6) & 3); }
template <int SNW>
__device__ __forceinline__ int tile_n0(int tid = threadIdx.x) { return Cfg<SNW>::SNN * (tid >> 8); }
// acc[n] (+)= sgn * As[rows, :] Bs[16 (n0 + n).., :]^T.  LOWER: Bs is
// lower triangular and only its lower part is meaningful (the diagonal
// factor's L^{-1} image, left in LDS): entries k > row read as 0.
template <int SNW, bool NEG, bool LOWER = false>
__device__ __forceinline__ void tile_mma(const double* As, const double* Bs, acc_t (&acc)[Cfg<SNW>::SNN],
                                         int tid = threadIdx.x) {
  const int lane = tid & 63;
  const int arow = tile_r0(tid) + (lane & 15), n0 = tile_n0<SNW>(tid);
#pragma unroll 4
  for (int s = 0; s < 16; ++s) {
    const int k = 4 * s + (lane >> 4);
    const double a = NEG ? -As[arow * DS + k] : As[arow * DS + k];
#pragma unroll
    for (int n = 0; n < Cfg<SNW>::SNN; ++n) {
      const int brow = 16 * (n0 + n) + (lane & 15);
      const double b = Bs[brow * DS + k];
      acc[n] = MF::mma(a, LOWER ? (k <= brow ? b : 0.0) : b, acc[n]);
    }
  }
}
}  // namespace

template <int SNW>
__global__ __launch_bounds__(64 * SNW) __attribute__((amdgpu_waves_per_eu(2))) void ldlt_small_kernel(double* __restrict__ K, int64_t ld, int N,
                                                         double* __restrict__ D, double* __restrict__ Linv,
                                                         double* __restrict__ W, int* __restrict__ info, int64_t sK,
                                                         int64_t sD, int64_t sL, int64_t sW,
                                                         const double* __restrict__ K0) {
  constexpr int SFR = Cfg<SNW>::SFR, SNN = Cfg<SNW>::SNN;
  __shared__ __attribute__((aligned(16))) double smem[2 * 64 * DS + 64];
  const int64_t qp = blockIdx.x;
  K += qp * sK;
  if (K0) K0 += qp * sK;  // the assembled matrix: block column 0's steps read it (first touch), L goes to K
  D += qp * sD;
  Linv += qp * sL;
  W += qp * sW;  // N x 64 row-major: the current block column's W = L D
  const int lane = threadIdx.x & 63;
  const int r0 = tile_r0(), n0 = tile_n0<SNW>();
  double* As = smem;
  double* Bs = smem + 64 * DS;
  const int nblk = (N + 63) / 64;
  auto nrows = [&](int c) { return N - 64 * c < 64 ? N - 64 * c : 64; };
  for (int J = 0; J < nblk; ++J) {
    const int J0 = 64 * J;
    const double* KS = (J == 0 && K0) ? K0 : K;  // where this step's not yet updated tiles are read
    diag64_body<false, false, double, false, SNW>(K, ld, J0, nrows(J), D, Linv + (int64_t)J * 64 * 64, info, smem,
                                                  smem + 64 * DS, smem + 2 * 64 * DS, nullptr, NoHook(), KS);
    if (J == nblk - 1) break;
    __syncthreads();  // diag64_body's L, D, L^{-1} stores are visible to the workgroup
    // ---- TRSM of the chunks below (block J is full: J0 + 64 < N), with
    // L_JJ^{-1} and the pivots straight from diag64_body's LDS images (X in
    // Bs, lower part; dsh) -- no global round trip on the chain
    double v[SFR], u[SFR];
    tile_fetch<SNW>(KS + (int64_t)(J0 + 64) * ld + J0, ld, nrows(J + 1), v);
    const double* dsh = smem + 2 * 64 * DS;
    double rd[SNN];
#pragma unroll
    for (int n = 0; n < SNN; ++n) rd[n] = 1.0 / dsh[16 * (n0 + n) + (lane & 15)];
    for (int c = J + 1; c < nblk; ++c) {
      const int rows = nrows(c);
      tile_put<SNW>(As, rows, v);
      __syncthreads();
      if (c + 1 < nblk) tile_fetch<SNW>(KS + (int64_t)(64 * (c + 1)) * ld + J0, ld, nrows(c + 1), v);
      acc_t acc[SNN];
#pragma unroll
      for (int n = 0; n < SNN; ++n) acc[n] = (acc_t){0.0, 0.0, 0.0, 0.0};
      tile_mma<SNW, false, true>(As, Bs, acc);
#pragma unroll
      for (int n = 0; n < SNN; ++n) {
        const int col = 16 * (n0 + n) + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = r0 + MF::row(lane, g);
          if (row < rows) {
            W[(int64_t)(64 * c + row) * 64 + col] = acc[n][g];
            K[(int64_t)(64 * c + row) * ld + J0 + col] = acc[n][g] * rd[n];
          }
        }
      }
      __syncthreads();  // As / Bs reads done before the next tile is staged
    }
    // ---- trailing update of the lower triangle below block J, tile (c, q)
    // in row order (the next diagonal block first); L[c, J] staged once per
    // row of tiles
    int c = J + 1, q = J + 1;
    tile_fetch<SNW>(K + (int64_t)(64 * c) * ld + J0, ld, nrows(c), v);  // L[c, J]
    tile_fetch<SNW>(W + (int64_t)(64 * q) * 64, 64, nrows(q), u);       // W_q
    for (;;) {
      const int rows = nrows(c);
      if (q == J + 1) tile_put<SNW>(As, rows, v);
      tile_put<SNW>(Bs, nrows(q), u);
      // the target tile C: its loads stay in flight through the MFMA chain,
      // which accumulates -L W^T from zero; C is added at the end
      acc_t acc[SNN], cv[SNN];
      const bool diag = q == c;
      // this lane's elements: rows r0 + (lane >> 4) + 4g, columns 16 (n0 + n) + (lane & 15)
      const int64_t toff = (int64_t)(64 * c + r0 + (lane >> 4)) * ld + 64 * q + 16 * n0 + (lane & 15);
      double* Ct = K + toff;
      const double* Cs = KS + toff;  // (block column 0's step: the assembled matrix)
      const double* Ct0 = KS + (int64_t)(64 * c) * ld + 64 * q;
      const int64_t ld4 = 4 * ld;
#pragma unroll
      for (int n = 0; n < SNN; ++n) {
        const int col = 16 * (n0 + n) + (lane & 15);
        acc[n] = (acc_t){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = r0 + MF::row(lane, g);
          const bool in = row < rows && (!diag || col <= row);
          cv[n][g] = *(in ? Cs + g * ld4 + 16 * n : Ct0);  // (out-of-tile lanes: a valid dummy address)
        }
      }
      __syncthreads();
      // next tile's operands
      int cn = c, qn = q + 1;
      if (qn > cn) {
        ++cn;
        qn = J + 1;
      }
      const bool more = cn < nblk;
      if (more) {
        if (qn == J + 1) tile_fetch<SNW>(K + (int64_t)(64 * cn) * ld + J0, ld, nrows(cn), v);
        tile_fetch<SNW>(W + (int64_t)(64 * qn) * 64, 64, nrows(qn), u);
      }
      tile_mma<SNW, true>(As, Bs, acc);
#pragma unroll
      for (int n = 0; n < SNN; ++n) {
        const int col = 16 * (n0 + n) + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = r0 + MF::row(lane, g);
          if (row < rows && (!diag || col <= row)) Ct[g * ld4 + 16 * n] = cv[n][g] + acc[n][g];
        }
      }
      __syncthreads();  // As / Bs free; the tile's stores visible to the next diagonal factor
      if (!more) break;
      c = cn;
      q = qn;
    }
  }
}

// ---------------------------------------------------------------------------
// Left-looking variant (round 4): every tile of block column J is formed
// ONCE, in registers, from the assembled matrix and the finished columns,
//   T(c, J) = A(c, J) - sum_{K<J} L(c, K) (L(J, K) D_K)^T,     c >= J,
// then factored (c = J: diag64_body, handed over through LDS) or solved
// (c > J: L(c, J) = T X_J^T / D_J), and L stored once.  Against the
// right-looking kernel above: no read-modify-write of trailing tiles and no W
// buffer -- the loads of a step are finished L tiles, independent of the
// MFMAs, so they are prefetched two tiles ahead.  Same tile MFMAs (16x16x4
// f64 over 64-wide k blocks); the sums over K are accumulated in registers
// before the subtraction (1e-16-level rounding differences against the
// right-looking order).  Columns c > J are formed CM tiles at a time.
// LDS: P0/P1 A operands (alternating), P2/P3 B operands (P3 doubles as
// diag64_body's X = L_JJ^{-1}, read by the TRSMs), D of every finished column.
// EXP (kbench attribution only, results meaningless when set): bit 0 skips
// the diagonal factors, bit 1 the MFMAs, bit 2 the operand tile loads
template <int SNW, int CM, int EXP = 0>
__global__ __launch_bounds__(64 * SNW) __attribute__((amdgpu_waves_per_eu(2))) void ldlt_small_left_kernel(
    double* __restrict__ K, int64_t ld, int N, double* __restrict__ D, double* __restrict__ Linv,
    int* __restrict__ info, int64_t sK, int64_t sD, int64_t sL, const double* __restrict__ K0) {
  constexpr int SFR = Cfg<SNW>::SFR, SNN = Cfg<SNW>::SNN, TB = 64 * DS;
  __shared__ __attribute__((aligned(16))) double smem[4 * TB + 64 + IPMZ_SMALL_NMAX];
  const int64_t qp = blockIdx.x;
  K += qp * sK;
  D += qp * sD;
  Linv += qp * sL;
  const double* KS = K0 ? K0 + qp * sK : K;  // the assembled matrix: every entry read once
  // buffer offsets opaque to the compiler (uniform SGPRs): every LDS access is
  // then one base VGPR + an immediate offset; with constant offsets past the
  // 64 KB immediate range the compiler materialised one VGPR per unrolled
  // access and spilled
  int o1 = TB;
  asm volatile("" : "+s"(o1));
  double* const P0 = smem;
  double* const P1 = smem + o1;
  double* const P2 = smem + 2 * o1;
  double* const P3 = smem + 3 * o1;
  double* const dsh = smem + 4 * o1;
  double* const dall = dsh + 64;
  const int nblk = (N + 63) / 64;
  auto nrows = [&](int c) { return N - 64 * c < 64 ? N - 64 * c : 64; };
  auto Lt = [&](int c, int Kb) { return K + (int64_t)(64 * c) * ld + 64 * Kb; };  // tile L(c, Kb)
  int abuf = 0;  // P0 / P1 alternation of the A operands (one barrier per tile)
  for (int J = 0; J < nblk; ++J) {
    const int J0 = 64 * J, b = nrows(J);
    // the thread index laundered per block column: nothing lane-dependent is
    // hoisted out of this loop (the hoisted diag64 / tile addresses of all
    // phases at once spilled)
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, r0 = tile_r0(tid), n0 = tile_n0<SNW>(tid);
    // acc <- this lane's elements of A(c, J) (lower part when c == J; lanes
    // outside read a valid dummy address and are never used)
    auto load_a = [&](int c, int J, acc_t(&acc)[SNN], int t) {
      const int rows = nrows(c), ln = t & 63, rr0 = tile_r0(t), nn0 = tile_n0<SNW>(t);
      const double* base = KS + (int64_t)(64 * c + rr0 + (ln >> 4)) * ld + 64 * J + 16 * nn0 + (ln & 15);
#pragma unroll
      for (int n = 0; n < SNN; ++n) {
        const int col = 16 * (nn0 + n) + (ln & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = rr0 + MF::row(ln, g);
          const bool in = row < rows && (c != J || col <= row);
          acc[n][g] = *(in ? base + (int64_t)g * 4 * ld + 16 * n : KS);
        }
      }
    };
    __syncthreads();  // the previous column's TRSM reads of P0..P3 and its dall store done
    // ---- T(J, J), then its factor
    if (J == 0) {
      if constexpr (!(EXP & 1))
      diag64_body<false, false, double, false, SNW>(K, ld, 0, b, D, Linv, info, P0, P3, dsh, nullptr, NoHook(), KS, tid);
    } else {
      acc_t acc[SNN];
      load_a(J, J, acc, tid);
      double va[SFR], vb[SFR];
      tile_fetch<SNW>(Lt(J, 0), ld, b, va, tid);
      if (J > 1) tile_fetch<SNW>(Lt(J, 1), ld, b, vb, tid);
      auto step = [&](int Kb, double(&v)[SFR]) {
        double* pa = (Kb & 1) ? P1 : P0;
        double* pb = (Kb & 1) ? P3 : P2;
        tile_put<SNW>(pa, b, v, tid);
        tile_put_scaled<SNW>(pb, b, v, dall[64 * Kb + lane], tid);
        __syncthreads();
        if (Kb + 2 < J && !(EXP & 4)) tile_fetch<SNW>(Lt(J, Kb + 2), ld, b, v, tid);
        if constexpr (!(EXP & 2)) tile_mma<SNW, true>(pa, pb, acc, tid);
      };
      for (int Kb = 0; Kb < J; Kb += 2) {
        step(Kb, va);
        if (Kb + 1 < J) step(Kb + 1, vb);
      }
      __syncthreads();  // P0..P3 reads done: T goes to P0 as diag64_body's M
#pragma unroll
      for (int n = 0; n < SNN; ++n) {
        const int col = 16 * (n0 + n) + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = r0 + MF::row(lane, g);
          P0[row * DS + col] = (row < b && col <= row) ? acc[n][g] : (row == col ? 1.0 : 0.0);
        }
      }
      if constexpr (!(EXP & 1))
      diag64_body<false, false, double, true, SNW>(K, ld, J0, b, D, Linv + (int64_t)J * 64 * 64, info, P0, P3, dsh,
                                                   nullptr, NoHook(), nullptr, tid);
    }
    if (J == nblk - 1) break;
    __syncthreads();  // diag64_body's write-back done reading P0; X (P3) and dsh final
    if (tid < 64) dall[J0 + tid] = dsh[tid];
    double rd[SNN];
#pragma unroll
    for (int n = 0; n < SNN; ++n) rd[n] = 1.0 / dsh[16 * (n0 + n) + (lane & 15)];
    // ---- T(c, J), c > J, CM tiles at a time: the stream of operand tiles is
    // (for each K < J) L(J, K) -> P2 scaled by D_K, then L(c, K) for the
    // chunk's c, each followed by its MFMAs
    for (int cb = J + 1; cb < nblk; cb += CM) {
      const int nc = nblk - cb < CM ? nblk - cb : CM;
      asm volatile("" : "+v"(tid));  // (again: nothing hoisted out of the chunk loop)
      const int lane = tid & 63, r0 = tile_r0(tid), n0 = tile_n0<SNW>(tid);
      acc_t acc[CM][SNN];
#pragma unroll
      for (int ci = 0; ci < CM; ++ci)
        if (ci < nc) load_a(cb + ci, J, acc[ci], tid);
      const int S = J * (nc + 1);
      auto src = [&](int s, double(&v)[SFR]) {
        if constexpr ((EXP & 4) != 0) return;
        const int Kb = s / (nc + 1), t = s - Kb * (nc + 1);
        if (t == 0) tile_fetch<SNW>(Lt(J, Kb), ld, 64, v, tid);
        else tile_fetch<SNW>(Lt(cb + t - 1, Kb), ld, nrows(cb + t - 1), v, tid);
      };
      auto step = [&](int s, double(&v)[SFR]) {
        const int Kb = s / (nc + 1), t = s - Kb * (nc + 1);
        if (t == 0) {
          __syncthreads();  // the previous K's MFMAs done reading P2
          tile_put_scaled<SNW>(P2, 64, v, dall[64 * Kb + lane], tid);
          if (s + 2 < S) src(s + 2, v);
          return;
        }
        double* pa = abuf ? P1 : P0;
        abuf ^= 1;
        tile_put<SNW>(pa, nrows(cb + t - 1), v, tid);
        __syncthreads();
        if (s + 2 < S) src(s + 2, v);
#pragma unroll
        for (int ci = 0; ci < CM; ++ci)
          if (ci == t - 1 && !(EXP & 2)) tile_mma<SNW, true>(pa, P2, acc[ci], tid);
      };
      if (S > 0) {
        double va[SFR], vb[SFR];
        src(0, va);
        src(1, vb);  // S >= 2 (a B tile and at least one A tile per K)
        for (int s = 0; s < S; s += 2) {
          step(s, va);
          if (s + 1 < S) step(s + 1, vb);
        }
      }
      // ---- TRSM: L(c, J) = T(c, J) X_J^T / D_J (T through P0 / P1 as the A operand)
#pragma unroll
      for (int ci = 0; ci < CM; ++ci) {
        if (ci >= nc) break;
        const int c = cb + ci, rows = nrows(c);
        double* pa = abuf ? P1 : P0;
        abuf ^= 1;
#pragma unroll
        for (int n = 0; n < SNN; ++n) {
          const int col = 16 * (n0 + n) + (lane & 15);
#pragma unroll
          for (int g = 0; g < 4; ++g) pa[(r0 + MF::row(lane, g)) * DS + col] = acc[ci][n][g];
        }
        __syncthreads();
        acc_t l[SNN];
#pragma unroll
        for (int n = 0; n < SNN; ++n) l[n] = (acc_t){0.0, 0.0, 0.0, 0.0};
        if constexpr (!(EXP & 2)) tile_mma<SNW, false, true>(pa, P3, l, tid);
#pragma unroll
        for (int n = 0; n < SNN; ++n) {
          const int col = 16 * (n0 + n) + (lane & 15);
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int row = r0 + MF::row(lane, g);
            if (row < rows) K[(int64_t)(64 * c + row) * ld + J0 + col] = l[n][g] * rd[n];
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Wave-specialized left-looking factor, N <= 64 NB <= 320 (C4's N = 320:
// NB = 5).  The kernel above runs the diagonal factors -- the chain, ~14 us
// per 64 x 64 block, one wave busy -- with the other seven waves waiting.
// Here waves 0..3 (the chain group) only factor diagonal blocks (diag64_body,
// NW = 4), while waves 4..7 (the bulk group) form the next tiles in the
// chain's shadow:
//   window J   chain: diag(J) (WS_NBAR barriers)
//              bulk : TRSM(c, J-1) of the chunks c > J (X_{J-1} is still in
//                     LDS until diag(J) writes X, after its third barrier),
//                     then T(c, J) = A(c, J) - sum_{K<J} L(c, K) W(J, K)^T,
//                     c > J, and the next diagonal tile minus its terms K < J,
//                     one tile of MFMAs per barrier interval, padded to WS_NBAR
//   transition bulk : TRSM(J+1, J) -> L(J+1, J), its W = L D into LDS (T1),
//                     the last term of T(J+1, J+1) -> LDS as the next M (T2)
// Both groups run the same barriers (raw counts match by construction; see
// ws_window_bars).  The bulk group keeps its tiles TRANSPOSED in registers --
// wave 4 + w owns columns 16 w .. 16 w + 15 of every T^T (rows of L) -- so a
// TRSM reads its T straight from registers (the accumulator layout of a
// 16 x 16 block is the B fragment of the next NN product) and its L operand
// rows come from global memory into registers (k order permuted so each lane
// loads 32 contiguous bytes); only W = L D is staged in LDS.
constexpr int WS_NBAR = 10;  // barriers of one diag64_body call (clkbuf == nullptr)
// kbench attribution (CLK instantiation only): s_memtime stamps of QP 0,
// chain group [0, 64), bulk group [64, 128)
__device__ unsigned long long ws_clk[128];
__host__ __device__ constexpr int ws_window_bars(int NB, int J) {
  // leftover TRSMs + per K < J: a staging interval and one per tile c > J
  // (the next diagonal tile shares tile J+1's interval: the same L rows)
  return J == 0 || J + 1 >= NB ? 0 : (NB - J - 1) + J * (1 + (NB - J - 1));
}
__host__ __device__ constexpr bool ws_schedule_fits(int NB) {
  for (int J = 0; J < NB; ++J)
    // (two intervals left for the transition's first TRSM rows; leftovers before diag's X write)
    if (ws_window_bars(NB, J) > WS_NBAR - 2 || (J >= 1 && NB - J - 1 > 3)) return false;
  return true;
}
static_assert(ws_schedule_fits(2) && ws_schedule_fits(3) && ws_schedule_fits(4) && ws_schedule_fits(5), "WS schedule");

template <int NB, bool CLK = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void ldlt_small_ws_kernel(
    double* __restrict__ K, int64_t ld, int N, double* __restrict__ D, double* __restrict__ Linv,
    int* __restrict__ info, int64_t sK, int64_t sD, int64_t sL, const double* __restrict__ K0) {
  constexpr int TB = 64 * DS;
  __shared__ __attribute__((aligned(16))) double smem[4 * TB + 64 + 64 * NB];
  const int64_t qp = blockIdx.x;
  K += qp * sK;
  D += qp * sD;
  Linv += qp * sL;
  const double* KS = K0 ? K0 + qp * sK : K;  // the assembled matrix: every entry read once
  int o1 = TB;  // (opaque offsets: one base VGPR + immediates per LDS access, see above)
  asm volatile("" : "+s"(o1));
  double* const M = smem;             // the next diagonal tile (chain input)
  double* const W1 = smem + o1;       // W(J+1, K) = L(J+1, K) D_K (bulk; the transition's W(J+1, J))
  double* const W0 = smem + 2 * o1;   // W(J, K) (bulk)
  double* const X = smem + 3 * o1;    // L_JJ^{-1} (chain output, read by the TRSMs)
  double* const dsh = smem + 4 * o1;  // D_J (chain)
  double* const dall = dsh + 64;      // D of every finished column
  auto nrows = [&](int c) { return N - 64 * c < 64 ? N - 64 * c : 64; };
  __shared__ unsigned long long clk_sh[CLK ? 128 : 1];  // (stamps in LDS: no registers held)
  auto stamp = [&](int slot) {
    if constexpr (CLK)
      clk_sh[slot] = __builtin_amdgcn_s_memtime();  // (every lane: no branch)
  };
  if ((threadIdx.x >> 6) < 4) {
    // ---- chain group: diag(J), then the two transition barriers
    for (int J = 0; J < NB; ++J) {
      int tid = threadIdx.x;
      asm volatile("" : "+v"(tid));
      const int b = nrows(J);
      stamp(3 * J);
      // L^{-1} of block J-1 (still in X) is written by waves 1..3 while wave 0
      // runs diag(J)'s first column pass -- off the transition's critical path
      auto linv_prev = [&]() {
        double* dst = Linv + (int64_t)(J - 1) * 64 * 64;
        // the lower triangle only, to the end of the diagonal's 32-byte
        // sector: the batched solve (trsv_small.h) never reads above the
        // diagonal, and whole sectors of zeros need no HBM write
        for (int idx = tid - 64; idx < 64 * 64; idx += 192) {
          const int rr = idx >> 6, cc = idx & 63;
          if (cc <= (rr | 3)) dst[idx] = cc > rr ? 0.0 : X[rr * DS + cc];  // (block J-1 < NB-1: full)
        }
      };
      if (J == 0)
        diag64_body<false, false, double, false, 4, NoHook, false, NoHook, 1>(K, ld, 0, b, D, Linv, info, M, X, dsh, nullptr,
                                                                   NoHook(), KS, tid);
      else if (J < NB - 1)
        diag64_body<false, false, double, true, 4, NoHook, false, decltype(linv_prev), 1>(K, ld, 64 * J, b, D, Linv, info, M, X, dsh,
                                                                  nullptr, NoHook(), nullptr, tid, linv_prev);
      else  // the last block writes its own L^{-1}
        diag64_body<false, false, double, true, 4, NoHook, true, decltype(linv_prev), 1>(K, ld, 64 * J, b, D, Linv + (int64_t)J * 64 * 64, info,
                                                                 M, X, dsh, nullptr, NoHook(), nullptr, tid, linv_prev);
      stamp(3 * J + 1);
      if (J == NB - 1) break;
      if (tid < 64) dall[64 * J + tid] = dsh[tid];
      __syncthreads();  // T1
      __syncthreads();  // T2: M holds T(J+1, J+1)
      stamp(3 * J + 2);
    }
    if constexpr (CLK)
      if (blockIdx.x == 0 && threadIdx.x < 64) ws_clk[threadIdx.x] = clk_sh[threadIdx.x];
    return;
  }
  // ---- bulk group: wave 4 + w owns rows r = 16 w .. 16 w + 15 of every L
  // tile, i.e. columns r of every T^T
  acc_t T[NB - 1][4];  // T^T(c, .), slot c - 1: blocks jb (rows j = 16 jb + q + 4 g)
  acc_t PT[4];         // the next diagonal tile, transposed
  // A(c, J)^T (lower part for the diagonal tile c == J); rows r past the matrix read as 0
  // (32-bit element offsets from the QP's base: one VGPR per address, immediate column offsets)
  const unsigned ldu = (unsigned)ld;
  // 4 x 4 transpose across the lane groups q = l >> 4 (v_permlane32_swap,
  // then v_permlane16_swap, per 32-bit half): u[t] of group q -> u[q] of group t
  auto transpose4 = [&](double(&u)[4]) {
    unsigned lo[4], hi[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      lo[t] = __double2loint(u[t]);
      hi[t] = __double2hiint(u[t]);
    }
    auto sw = [](unsigned(&v)[4], int i, int j, bool s32) {
      const auto r = s32 ? __builtin_amdgcn_permlane32_swap(v[i], v[j], false, false)
                         : __builtin_amdgcn_permlane16_swap(v[i], v[j], false, false);
      v[i] = r[0];
      v[j] = r[1];
    };
    sw(lo, 0, 2, true), sw(lo, 1, 3, true), sw(lo, 0, 1, false), sw(lo, 2, 3, false);
    sw(hi, 0, 2, true), sw(hi, 1, 3, true), sw(hi, 0, 1, false), sw(hi, 2, 3, false);
#pragma unroll
    for (int t = 0; t < 4; ++t) u[t] = __hiloint2double(hi[t], lo[t]);
  };
  // A(c, J)^T (lower part for the diagonal tile c == J); rows r past the
  // matrix read as 0.  Each lane loads 32 contiguous bytes per 16-column
  // block (two 16-byte loads instead of four 8-byte ones) and the lane groups
  // exchange them into the accumulator layout.
  auto load_at = [&](int c, int J, acc_t(&a)[4], int tid) {
    const int l = tid & 63, q = l >> 4, r = 16 * ((tid >> 6) - 4) + (l & 15), rows = nrows(c);
    const double* src = KS + ((unsigned)(64 * c + (r < rows ? r : 0)) * ldu + 64 * J + 4 * q);
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      const double2 x0 = *reinterpret_cast<const double2*>(src + 16 * jb);
      const double2 x1 = *reinterpret_cast<const double2*>(src + 16 * jb + 2);
      double u[4] = {x0.x, x0.y, x1.x, x1.y};  // A[r][16 jb + 4 q + t]
      transpose4(u);                           // A[r][16 jb + q + 4 g]
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int j = 16 * jb + q + 4 * g;
        const bool in = r < rows && (c != J || j <= r);  // (the upper part of A(J, J) is read, not used)
        a[jb][g] = in ? u[g] : 0.0;
      }
    }
  };
  // this lane's L(c, Kb) row r, columns 16 u + 4 q + t (the k order of the
  // accumulation MFMAs): 32 contiguous bytes per u
  auto load_bf = [&](int c, int Kb, double(&bf)[16], int tid) {
    const int l = tid & 63, q = l >> 4, r = 16 * ((tid >> 6) - 4) + (l & 15), rows = nrows(c);
    const double2* src =
        reinterpret_cast<const double2*>(K + ((unsigned)(64 * c + (r < rows ? r : 0)) * ldu + 64 * Kb + 4 * q));
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double2 x0 = src[8 * u], x1 = src[8 * u + 1];
      bf[4 * u] = x0.x;
      bf[4 * u + 1] = x0.y;
      bf[4 * u + 2] = x1.x;
      bf[4 * u + 3] = x1.y;
    }
  };
  // a^T -= Ls (bf D_Kb)^T over one 64-wide k block: the plain L copy in LDS
  // (rows j) against this lane's L rows scaled by the pivots (W = L D)
  auto mma_acc = [&](acc_t(&a)[4], const double* Ls, const double(&bf)[16], int Kb, int tid) {
    const int l = tid & 63, q = l >> 4;
    const double* base = Ls + (l & 15) * DS + 4 * q;
    const double* dk = dall + 64 * Kb + 4 * q;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const double b = bf[4 * u + t] * dk[16 * u + t];
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) a[jb] = MF::mma(-base[16 * jb * DS + 16 * u + t], b, a[jb]);
        __builtin_amdgcn_sched_barrier(0);  // (bounds the LDS operands in flight: registers)
      }
  };
  // L^T = diag(1 / d) X T^T: X (lower, LDS) against T^T's blocks as B
  // fragments; lt[ib] rows i = 16 ib + q + 4 g; d: the pivots in LDS
  // rows [ib0, ib1) of it only (the transition's TRSM starts in the window,
  // as soon as those rows of X_J are final)
  auto trsm_rows = [&](const acc_t(&a)[4], acc_t(&lt)[4], const double* d, int tid, auto ib0c, auto ib1c) {
    constexpr int IB0 = decltype(ib0c)::value, IB1 = decltype(ib1c)::value;
    const int l = tid & 63, q = l >> 4;
    const double* xr = X + (l & 15) * DS + q;
#pragma unroll
    for (int ib = IB0; ib < IB1; ++ib) lt[ib] = (acc_t){0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int jb = 0; jb < IB1; ++jb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
#pragma unroll
        for (int ib = (jb > IB0 ? jb : IB0); ib < IB1; ++ib)
          lt[ib] = MF::mma(xr[16 * ib * DS + 16 * jb + 4 * g], a[jb][g], lt[ib]);
        if (g == 3) __builtin_amdgcn_sched_barrier(0);  // (per block column: registers; chains interleave)
      }
#pragma unroll
    for (int ib = IB0; ib < IB1; ++ib)
#pragma unroll
      for (int g = 0; g < 4; ++g) lt[ib][g] *= fast_rcp(d[16 * ib + q + 4 * g]);
  };
  auto trsm = [&](const acc_t(&a)[4], acc_t(&lt)[4], const double* d, int tid) {
    trsm_rows(a, lt, d, tid, std::integral_constant<int, 0>{}, std::integral_constant<int, 4>{});
  };
  // L(c, J) rows r of this wave: transposed through the wave's own rows of a
  // free LDS tile, then stored a whole 512-byte row per instruction (the
  // register layout would store 32-byte pieces of 16 rows per instruction)
  auto put_l = [&](const acc_t(&lt)[4], double* buf, int tid) {
    const int l = tid & 63, q = l >> 4, r = 16 * ((tid >> 6) - 4) + (l & 15);
#pragma unroll
    for (int ib = 0; ib < 4; ++ib)
#pragma unroll
      for (int g = 0; g < 4; ++g) buf[r * DS + 16 * ib + q + 4 * g] = lt[ib][g];
  };
  auto rows_out = [&](int c, int J, const double* buf, int tid) {  // this wave's rows of buf -> L(c, J)
    // two rows per instruction, 16 bytes per lane (half the memory instructions)
    const int l = tid & 63, w = (tid >> 6) - 4, rows = nrows(c), h = l >> 5, col = 2 * (l & 31);
    unsigned o = (unsigned)(64 * c + 16 * w + h) * ldu + 64 * J + col;
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      const int r = 16 * w + i + h;
      if (r < rows) {
        double2 x;
        x.x = buf[r * DS + col];
        x.y = buf[r * DS + col + 1];
        *reinterpret_cast<double2*>(K + o) = x;
      }
      o += 2 * ldu;
      if ((i & 7) == 6) __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto store_l = [&](int c, int J, const acc_t(&lt)[4], double* buf, int tid) {
    put_l(lt, buf, tid);
    rows_out(c, J, buf, tid);
  };
  // plain copies of L(J, Kb) -> W0 and L(J+1, Kb) -> W1 (256 threads; rows
  // past the matrix zero): loads into v, then the LDS stores
  // (W1P = false: only the W0 part -- W1 already holds its tile)
  // (16 bytes per lane: two rows per instruction)
  auto stage_load = [&](int J, int Kb, double2(&v)[16], bool w1p, int tid) {
    const int t = tid - 256, col = 2 * (t & 31), rows1 = nrows(J + 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = (t >> 5) + 8 * i;
      v[i] = *reinterpret_cast<const double2*>(K + ((unsigned)(64 * J + r) * ldu + 64 * Kb + col));  // (J < NB-1: full)
      if (w1p)
        v[8 + i] = *reinterpret_cast<const double2*>(
            K + ((unsigned)(64 * (J + 1) + (r < rows1 ? r : 0)) * ldu + 64 * Kb + col));
    }
  };
  auto stage_put = [&](const double2(&v)[16], int J, bool w1p, int tid) {
    const int t = tid - 256, col = 2 * (t & 31), rows1 = nrows(J + 1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = (t >> 5) + 8 * i;
      W0[r * DS + col] = v[i].x;
      W0[r * DS + col + 1] = v[i].y;
      if (w1p) {
        W1[r * DS + col] = r < rows1 ? v[8 + i].x : 0.0;
        W1[r * DS + col + 1] = r < rows1 ? v[8 + i].y : 0.0;
      }
    }
  };
  static_for<NB>([&](auto jc) {
    constexpr int J = decltype(jc)::value;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // nothing lane-dependent hoisted across windows
    int nb = 0;
    // raw barrier: this wave's LDS operations retired, its global loads and
    // stores stay in flight; FULL (__syncthreads): the stores complete too,
    // where another interval reads them next
    auto bar = [&](bool full) {
      if (full) {
        __syncthreads();
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);  // (nothing scheduled across intervals: registers)
      ++nb;
      stamp(64 + 13 * J + nb);
    };
    stamp(64 + 13 * J);
    // ======== window J (the chain factors block J)
    if constexpr (J >= 1) rows_out(J, J - 1, W0, tid);  // the transition's L(J, J-1), transposed into W0
    if constexpr (J == 0) {
      static_for<NB - 1>([&](auto cc) { load_at(decltype(cc)::value + 1, 0, T[decltype(cc)::value], tid); });
      if constexpr (NB > 1) load_at(1, 1, PT, tid);
    } else if constexpr (J + 1 < NB) {
      constexpr int NL = NB - J - 1;  // leftover TRSMs of column J-1 = tiles c = J+1 .. NB-1 per K
      // the first K step's operands, loaded under the leftovers: L(J, 0)
      // (earlier windows) and L(J+1, 0) -- for J = 1 that tile is the first
      // leftover's own result, transposed straight into W1 below
      double2 stg[16];
      double bfa[16], bfb[16];
      if constexpr (J == 1) {
        // L(1, 0) is the tile the other waves are storing just above (no
        // barrier in between: a global load here could return the old
        // contents of K); W0 still holds it in the staging layout
        const int t = tid - 256, col = 2 * (t & 31);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int r = (t >> 5) + 8 * i;
          stg[i].x = W0[r * DS + col];
          stg[i].y = W0[r * DS + col + 1];
        }
      } else {
        stage_load(J, 0, stg, true, tid);
      }
      // X_{J-1} stays intact until diag(J)'s 4th interval (NL <= 3)
      static_for<NL>([&](auto cc) {
        constexpr int c = J + 1 + decltype(cc)::value;
        acc_t lt[4];
        trsm(T[c - 1], lt, dall + 64 * (J - 1), tid);
        if constexpr (J == 1) stamp(20 + 3 * decltype(cc)::value);
        // (W0 is restaged after the leftovers; W1 then holds L(2, 0) for J = 1)
        store_l(c, J - 1, lt, (J == 1 && c == 2) ? W1 : W0, tid);
        if constexpr (J == 1) stamp(21 + 3 * decltype(cc)::value);
        __builtin_amdgcn_sched_barrier(0);  // (register pressure: the next loads stay here)
        load_at(c, J, T[c - 1], tid);  // T(c, J) starts from A(c, J)
        if constexpr (J == 1) stamp(22 + 3 * decltype(cc)::value);
        bar(decltype(cc)::value == NL - 1);  // the K loop reads these L rows
      });
      asm volatile("" ::: "memory");
      load_at(J + 1, J + 1, PT, tid);
      // K loop, per Kb: S (W0, W1 staged), M1 (tile J+1 and the diagonal
      // tile: the same L rows), Mc (c = J+2 ..); each item's global operand is
      // loaded one interval ahead
      static_for<J>([&](auto kc) {
        constexpr int Kb = decltype(kc)::value;
        stage_put(stg, J, J > 1 || Kb > 0, tid);
        asm volatile("" ::: "memory");
        load_bf(J + 1, Kb, bfa, tid);
        bar(false);
        if constexpr (NL >= 2) load_bf(J + 2, Kb, bfb, tid);
        else if constexpr (Kb + 1 < J) stage_load(J, Kb + 1, stg, true, tid);
        if constexpr (J == 1) stamp(30);
        mma_acc(T[J], W0, bfa, Kb, tid);
        if constexpr (J == 1) stamp(31);
        mma_acc(PT, W1, bfa, Kb, tid);
        if constexpr (J == 1) stamp(32);
        bar(false);
        static_for<NL - 1>([&](auto cc) {
          constexpr int ci = decltype(cc)::value, c = J + 2 + ci;
          auto& cur = (ci % 2 == 0) ? bfb : bfa;
          auto& nxt = (ci % 2 == 0) ? bfa : bfb;
          if constexpr (c + 1 < NB) load_bf(c + 1, Kb, nxt, tid);
          else if constexpr (Kb + 1 < J) stage_load(J, Kb + 1, stg, true, tid);
          mma_acc(T[c - 1], W0, cur, Kb, tid);
          bar(false);
        });
      });
    }
    // rows 0..47 of L(J+1, J) in the window's 9th interval: X_J's block rows
    // 0..2 are final after diag(J)'s 8th barrier (its inverse tiles X_22,
    // X_20, X_21 in the 8th interval), D_J after the third column pass
    acc_t lt[4];
    if constexpr (J + 1 < NB) {
      while (nb < WS_NBAR - 2) bar(false);
      trsm_rows(T[J], lt, dsh, tid, std::integral_constant<int, 0>{}, std::integral_constant<int, 3>{});
    }
    while (nb < WS_NBAR) bar(false);
    // ======== transition: L(J+1, J) and the last term of T(J+1, J+1) -> M
    if constexpr (J + 1 < NB) {
      const int l = tid & 63, q = l >> 4, r = 16 * ((tid >> 6) - 4) + (l & 15), b = nrows(J + 1);
      // its last block row (X_J final after diag(J)'s last barrier)
      trsm_rows(T[J], lt, dsh, tid, std::integral_constant<int, 3>{}, std::integral_constant<int, 4>{});
      if constexpr (J == 1) stamp(33);
      put_l(lt, W0, tid);  // L(J+1, J) -> global from W0 in the next window's first interval
      if constexpr (J == 1) stamp(34);
#pragma unroll
      for (int ib = 0; ib < 4; ++ib)  // W(J+1, J) = L(J+1, J) D_J: this wave's rows r
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int i = 16 * ib + q + 4 * g;
          W1[r * DS + i] = lt[ib][g] * dsh[i];
        }
      stamp(64 + 13 * J + 11);
      __syncthreads();  // T1 (the chain's write-back of diag(J) done with M)
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        const double* wr = W1 + (16 * jb + (l & 15)) * DS + q;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int g = 0; g < 4; ++g) PT[jb] = MF::mma(-wr[16 * kb + 4 * g], lt[kb][g], PT[jb]);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int j = 16 * jb + q + 4 * g;
          M[r * DS + j] = (r < b && j <= r) ? PT[jb][g] : (r == j ? 1.0 : 0.0);
        }
      __syncthreads();  // T2 (also: L(J+1, J) stored before the next window reads it)
      stamp(64 + 13 * J + 12);
    }
  });
  if constexpr (CLK)
    if (blockIdx.x == 0 && threadIdx.x >= 256 && threadIdx.x < 320) ws_clk[threadIdx.x - 192] = clk_sh[threadIdx.x - 192];
}

// ---------------------------------------------------------------------------
// The same factor with TWO workgroups per QP, for batches that leave CUs
// idle (2B <= #CU: C4's 128 QPs per GPU at 8 GPUs; N = 320, B = 128: 194 ->
// 177 us -- the five 64-column diagonal blocks, ~15 us each, stay on one
// chain).  Role 0 carries the
// critical path -- the diagonal block J, the TRSM of every chunk below it and
// the trailing tiles of column J+1 (which hold the next diagonal block and
// the next TRSM's operands) -- and role 1, on another CU, the rest of the
// trailing update of step J (columns J+2..), in the shadow of role 0's next
// diagonal factor.  Hand-offs per step (sync.h protocol: write-through
// stores, vmcnt drain, barrier, one flag store; consumers poll and read with
// agent-scope loads):
//   LW[J]    role 0 -> 1: L(c, J) in K and W(c, J) (parity J & 1 of the
//            two W buffers) for every chunk c > J
//   DONE[J]  role 1 -> 0: step J's tiles of columns >= J+2 stored (role 0
//            needs column J+2 of them at step J+1)
// Each element keeps the single-workgroup kernel's arithmetic (the same MFMA
// tiles in the same order), so the factor is identical to it.
template <int SNW>
__global__ __launch_bounds__(64 * SNW) void ldlt_small_pair_kernel(double* __restrict__ K, int64_t ld, int N,
                                                              double* __restrict__ D, double* __restrict__ Linv,
                                                              double* __restrict__ W, int* __restrict__ info,
                                                              int64_t sK, int64_t sD, int64_t sL, int64_t sW,
                                                              unsigned* __restrict__ flags, unsigned* __restrict__ err,
                                                              const double* __restrict__ K0) {
  constexpr int SFR = Cfg<SNW>::SFR, SNN = Cfg<SNW>::SNN;
  __shared__ __attribute__((aligned(16))) double smem[2 * 64 * DS + 64];
  __shared__ unsigned sh_ok;
  const int64_t qp = blockIdx.x >> 1;
  const int role = blockIdx.x & 1;
  K += qp * sK;
  if (K0) K0 += qp * sK;  // block column 0's steps read the assembled matrix (not written by this launch)
  D += qp * sD;
  Linv += qp * sL;
  W += qp * sW;  // two N x 64 row-major buffers (parity of J): W = L D of block column J
  unsigned* LW = flags + qp * IPMZ_PAIR_FLAGS;
  unsigned* DONE = LW + IPMZ_PAIR_FLAGS / 2;
  const int lane = threadIdx.x & 63;
  const int r0 = tile_r0(), n0 = tile_n0<SNW>();
  double* As = smem;
  double* Bs = smem + 64 * DS;
  const int nblk = (N + 63) / 64;
  auto nrows = [&](int c) { return N - 64 * c < 64 ? N - 64 * c : 64; };
  auto Wj = [&](int J) { return W + (int64_t)(J & 1) * N * 64; };
  // tiles (c, q), c >= q, for q in [qlo, qhi], in row order, -= L(c, J) W_q^T;
  // operands of the next tile loaded while the current one computes.  All
  // global traffic agent-scope: L / W come from role 0, tiles of column J+2
  // go to it.
  auto trail = [&](int J, int qlo, int qhi) {
    if (qlo > qhi || qlo >= nblk) return;
    const double* Wb = Wj(J);
    double v[SFR], u[SFR];
    int c = qlo, q = qlo;
    tile_fetch_sc<SNW>(K + (int64_t)(64 * c) * ld + 64 * J, ld, nrows(c), v);  // L[c, J]
    tile_fetch_sc<SNW>(Wb + (int64_t)(64 * q) * 64, 64, nrows(q), u);           // W_q
    for (;;) {
      const int rows = nrows(c);
      if (q == qlo) tile_put<SNW>(As, rows, v);
      tile_put<SNW>(Bs, nrows(q), u);
      acc_t acc[SNN], cv[SNN];
      const bool diag = q == c;
      const int64_t toff = (int64_t)(64 * c + r0 + (lane >> 4)) * ld + 64 * q + 16 * n0 + (lane & 15);
      double* Ct = K + toff;
      const double* Cs = ((J == 0 && K0) ? K0 : K) + toff;  // block column 0's step: the assembled matrix
      const double* Ct0 = K + (int64_t)(64 * c) * ld + 64 * q;
      const int64_t ld4 = 4 * ld;
#pragma unroll
      for (int n = 0; n < SNN; ++n) {
        const int col = 16 * (n0 + n) + (lane & 15);
        acc[n] = (acc_t){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = r0 + MF::row(lane, g);
          const bool in = row < rows && (!diag || col <= row);
          cv[n][g] = ld_sc1(in ? Cs + g * ld4 + 16 * n : Ct0);
        }
      }
      __syncthreads();
      int cn = c, qn = q + 1;
      if (qn > cn || qn > qhi) {
        ++cn;
        qn = qlo;
      }
      const bool more = cn < nblk;
      if (more) {
        if (qn == qlo) tile_fetch_sc<SNW>(K + (int64_t)(64 * cn) * ld + 64 * J, ld, nrows(cn), v);
        tile_fetch_sc<SNW>(Wb + (int64_t)(64 * qn) * 64, 64, nrows(qn), u);
      }
      tile_mma<SNW, true>(As, Bs, acc);
#pragma unroll
      for (int n = 0; n < SNN; ++n) {
        const int col = 16 * (n0 + n) + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = r0 + MF::row(lane, g);
          if (row < rows && (!diag || col <= row)) st_sc1(Ct + g * ld4 + 16 * n, cv[n][g] + acc[n][g]);
        }
      }
      __syncthreads();
      if (!more) break;
      c = cn;
      q = qn;
    }
  };
  if (role == 1) {
    for (int J = 0; J + 2 < nblk; ++J) {
      if (!wait_flag(&LW[J], err, &sh_ok)) return;
      trail(J, J + 2, nblk - 1);
      publish(&DONE[J]);
    }
    return;
  }
  for (int J = 0; J < nblk; ++J) {
    const int J0 = 64 * J;
    const double* KS = (J == 0 && K0) ? K0 : K;  // where this step's not yet updated tiles are read
    // block J was last updated by this workgroup (column J+1 of step J-1) or
    // before the DONE[J-2] wait of step J-1 (agent-scope loads: LSC)
    diag64_body<false, true, double, false, SNW>(K, ld, J0, nrows(J), D, Linv + (int64_t)J * 64 * 64, info, smem,
                                                 smem + 64 * DS, smem + 2 * 64 * DS, nullptr, NoHook(), KS);
    if (J == nblk - 1) break;
    __syncthreads();
    // ---- TRSM of every chunk below, published for role 1
    double v[SFR];
    tile_fetch_sc<SNW>(KS + (int64_t)(J0 + 64) * ld + J0, ld, nrows(J + 1), v);
    const double* dsh = smem + 2 * 64 * DS;
    double* Wb = Wj(J);
    double rd[SNN];
#pragma unroll
    for (int n = 0; n < SNN; ++n) rd[n] = 1.0 / dsh[16 * (n0 + n) + (lane & 15)];
    for (int c = J + 1; c < nblk; ++c) {
      const int rows = nrows(c);
      tile_put<SNW>(As, rows, v);
      __syncthreads();
      if (c + 1 < nblk) tile_fetch_sc<SNW>(KS + (int64_t)(64 * (c + 1)) * ld + J0, ld, nrows(c + 1), v);
      acc_t acc[SNN];
#pragma unroll
      for (int n = 0; n < SNN; ++n) acc[n] = (acc_t){0.0, 0.0, 0.0, 0.0};
      tile_mma<SNW, false, true>(As, Bs, acc);
#pragma unroll
      for (int n = 0; n < SNN; ++n) {
        const int col = 16 * (n0 + n) + (lane & 15);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int row = r0 + MF::row(lane, g);
          if (row < rows) {
            st_sc1(&Wb[(int64_t)(64 * c + row) * 64 + col], acc[n][g]);
            st_sc1(&K[(int64_t)(64 * c + row) * ld + J0 + col], acc[n][g] * rd[n]);
          }
        }
      }
      __syncthreads();
    }
    publish(&LW[J]);
    // ---- column J+1 of the trailing update (the next diagonal block and the
    // next TRSM's operands), after role 1's step J-1 (it updated column J+1)
    if (J >= 1 && !wait_flag(&DONE[J - 1], err, &sh_ok)) return;
    trail(J, J + 1, J + 1);
  }
}

// 2B workgroups must all be resident at once to help: 256 VGPRs per lane x 8
// waves fill a CU, so one workgroup per CU -- 2B <= #CU (B = 128 at 8 GPUs)
bool small_pair_eligible(int B, int N) { return 2 * B <= device_cus() && N > 64 && N <= IPMZ_SMALL_NMAX; }

// Does ldlt_factor_small_batched launch the two-workgroup kernel (the only
// small factor with a cross-workgroup hand-off and an error word)?
bool small_pair_used(int kern, bool have_flags, int B, int N) {
  // a batch that leaves CUs idle: two workgroups per QP
  const bool pair_ok = have_flags && small_pair_eligible(B, N);
  const bool ws_ok = N > 64 && N <= 320;  // the wave-specialized left-looking factor beats the pair
  return pair_ok && (kern == IPMZ_BATCH_FACTOR_PAIR || (kern == IPMZ_BATCH_FACTOR_AUTO && !ws_ok));
}

hipError_t ldlt_factor_small_batched(double* K, int64_t ld, int N, double* D, double* Linv, double* W, int* info,
                                     hipStream_t st, const BatchStrides& bs) {
  if (N <= 0 || bs.B <= 0) return hipSuccess;
  const int kern = bs.small_kernel;
  if (small_pair_used(kern, bs.pflags != nullptr, bs.B, N)) {  // flags and error word zeroed here
    hipError_t e = hipMemsetAsync(bs.pflags, 0, ((size_t)bs.B * IPMZ_PAIR_FLAGS + 1) * sizeof(unsigned), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ldlt_small_pair_kernel<8>, dim3(2 * bs.B), dim3(64 * 8), 0, st, K, ld, N, D, Linv, W, info,
                       bs.sK, bs.sD, bs.sL, bs.sW, bs.pflags, bs.pflags + (size_t)bs.B * IPMZ_PAIR_FLAGS, bs.K0);
    return hipGetLastError();
  }
  if (kern == IPMZ_BATCH_FACTOR_ONE) {
    // 8 waves (two per SIMD) also when the batch leaves a CU per QP: 16 waves
    // measured slower (N = 320, B = 128: 249 vs 190 us)
    hipLaunchKernelGGL(ldlt_small_kernel<8>, dim3(bs.B), dim3(64 * 8), 0, st, K, ld, N, D, Linv, W, info, bs.sK,
                       bs.sD, bs.sL, bs.sW, bs.K0);
    return hipGetLastError();
  }
  // left-looking: wave-specialized up to N = 320 (C4: 1024 QPs 854 -> 706 us,
  // 128 QPs 195 -> 156 us against the right-looking factor), else the plain one
  const int nb = (N + 63) / 64;
  auto ws = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(bs.B), dim3(512), 0, st, K, ld, N, D, Linv, info, bs.sK, bs.sD, bs.sL, bs.K0);
  };
  if (nb == 5) ws(ldlt_small_ws_kernel<5>);
  else if (nb == 4) ws(ldlt_small_ws_kernel<4>);
  else if (nb == 3) ws(ldlt_small_ws_kernel<3>);
  else if (nb == 2) ws(ldlt_small_ws_kernel<2>);
  else
    hipLaunchKernelGGL((ldlt_small_left_kernel<8, 4>), dim3(bs.B), dim3(64 * 8), 0, st, K, ld, N, D, Linv, info,
                       bs.sK, bs.sD, bs.sL, bs.K0);
  return hipGetLastError();
}

// experiment entry (tools/kbench.cpp "smallv"): the one-workgroup factor with
// SNW = 4 waves (two workgroups -- two QPs -- per CU) or 8
hipError_t ldlt_factor_small_variant(int snw, double* K, int64_t ld, int N, double* D, double* Linv, double* W,
                                     int* info, hipStream_t st, const BatchStrides& bs) {
  if (snw >= 100) {  // 100 + EXP: the left-looking kernel's attribution variants
    auto l = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(bs.B), dim3(64 * 8), 0, st, K, ld, N, D, Linv, info, bs.sK, bs.sD, bs.sL, bs.K0);
    };
    switch (snw - 100) {
      case 1: l(ldlt_small_left_kernel<8, 4, 1>); break;
      case 2: l(ldlt_small_left_kernel<8, 4, 2>); break;
      case 3: l(ldlt_small_left_kernel<8, 4, 3>); break;
      case 4: l(ldlt_small_left_kernel<8, 4, 4>); break;
      case 6: l(ldlt_small_left_kernel<8, 4, 6>); break;
      case 7: l(ldlt_small_left_kernel<8, 4, 7>); break;
      default: l(ldlt_small_left_kernel<8, 4, 0>); break;
    }
  } else if (snw == 2) {  // the wave-specialized left-looking factor (N <= 320)
    const int nb = (N + 63) / 64;
    auto l = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(bs.B), dim3(512), 0, st, K, ld, N, D, Linv, info, bs.sK, bs.sD, bs.sL, bs.K0);
    };
    if (nb == 5 && (debug_inject_mask() & IPMZ_DEBUG_TRACE)) {
      l(ldlt_small_ws_kernel<5, true>);
      unsigned long long h[128];
      hipError_t e = hipMemcpyFromSymbol(h, HIP_SYMBOL(ws_clk), sizeof(h), 0, hipMemcpyDeviceToHost);
      if (e != hipSuccess) return e;
      const unsigned long long t0 = h[0];
      for (int J = 0; J < 5; ++J) {
        std::printf("ws J=%d chain: diag %llu..%llu T2 %llu | bulk: start %llu bars", J, h[3 * J] - t0, h[3 * J + 1] - t0,
                    J < 4 ? h[3 * J + 2] - t0 : 0ull, h[64 + 13 * J] - t0);
        for (int k = 1; k <= 10; ++k) std::printf(" %llu", h[64 + 13 * J + k] - t0);
        if (J < 4) std::printf(" | pre-T1 %llu T2 %llu", h[64 + 13 * J + 11] - t0, h[64 + 13 * J + 12] - t0);
        std::printf("\n");
      }
      std::printf("ws J=1 leftovers (trsm, store, load_at):");
      for (int k = 20; k < 29; ++k) std::printf(" %llu", h[k] - t0);
      std::printf(" | M1 %llu %llu %llu | transition trsm %llu store %llu\n", h[30] - t0, h[31] - t0, h[32] - t0,
                  h[33] - t0, h[34] - t0);
    } else if (nb == 5) l(ldlt_small_ws_kernel<5>);
    else if (nb == 4) l(ldlt_small_ws_kernel<4>);
    else if (nb == 3) l(ldlt_small_ws_kernel<3>);
    else if (nb == 2) l(ldlt_small_ws_kernel<2>);
    else return hipErrorInvalidValue;
  } else if (snw == 1)
    hipLaunchKernelGGL((ldlt_small_left_kernel<8, 4>), dim3(bs.B), dim3(64 * 8), 0, st, K, ld, N, D, Linv, info,
                       bs.sK, bs.sD, bs.sL, bs.K0);
  else if (snw == 4)
    hipLaunchKernelGGL(ldlt_small_kernel<4>, dim3(bs.B), dim3(64 * 4), 0, st, K, ld, N, D, Linv, W, info, bs.sK,
                       bs.sD, bs.sL, bs.sW, bs.K0);
  else
    hipLaunchKernelGGL(ldlt_small_kernel<8>, dim3(bs.B), dim3(64 * 8), 0, st, K, ld, N, D, Linv, W, info, bs.sK,
                       bs.sD, bs.sL, bs.sW, bs.K0);
  return hipGetLastError();
}

}  // namespace ipmz
