// Single-launch triangular solve with the LDL^T factor:
//   x = L^{-T} D^{-1} L^{-1} b   (LinearSolvers.cpp:44-74)
// on 128-row blocks, with the one hand-off per block that the chain of
// blocks needs reduced to ONE 128 x 128 mat-vec.
//
// Block J (rows J0 .. J0+128), X_J = L_JJ^{-1}:
//   forward : y_J = X_J (b_J - sum_{K<J-1} L_JK y_K) - M_J y_{J-1},
//             M_J = X_J L_{J,J-1}
//   backward: x_J = X_J^T (y_J / D_J - sum_{K>J+1} L_KJ^T x_K) - Q_J x_{J+1},
//             Q_J = (L_{J+1,J} X_J)^T
// X_J, X_J^T, M_J and Q_J are built once per factorization by
// solve_prep_kernel (fp64 MFMA, from the factor's 64 x 64 inverses) -- the
// same two solves of every Newton step (and every refinement solve of the
// mixed-precision path) reuse them.  Everything but the M_J / Q_J product is
// computed before the previous block's vector arrives, so a hand-off costs
// one poll plus one 128-wide dot product per row: 2 * N/128 hops per solve
// instead of 2 * N/64 hops of a 64 x 64 TRSV step each.
//
// Work distribution: the forward sweep (blocks 0..nb-1) and the backward
// sweep (nb-1..0) are two launches whose workgroups dequeue tickets from a
// device counter; a ticket only waits on lower tickets, which belong to
// running workgroups, so a grid cannot deadlock.
// The bulk L_JK y_K products stream the off-diagonal tiles in order, in
// pairs (512 threads x 2 x 32 elements = two 128 x 128 tiles in flight), a
// pair consumed as soon as its two block vectors are complete.  Readiness
// travels with the data: the vectors start as an all-ones bit pattern (a NaN
// payload arithmetic never produces) and are stored write-through (sc1), one
// aligned store per element (MI355X_MICROARCH.md, R2 granule), so ONE round
// of agent-scope loads both stages a vector and proves it complete.  Spins are bounded: on timeout ctrl[1]
// (SOLVE_ERR_WORD) is raised -- sticky, folded into the host's return codes.
#include "common.h"
#include "kernels.h"
#include "sync.h"

namespace ipmz {

// -DIPMZ_SOLVE_STAMPS: per forward block start / bulk done / critical wait / stored / y_{J-1} seen clocks (tools/kbench)
__device__ unsigned long long g_sstamp[2][256][6];
#ifdef IPMZ_SOLVE_STAMPS
#define SSTAMP(J, i) \
  if (tid == 0 && (J) < 256) g_sstamp[0][J][i] = __builtin_amdgcn_s_memrealtime()
#else
#define SSTAMP(J, i)
#endif
namespace {
constexpr int SB = IPMZ_SOLVE_BLOCK;  // rows per solve block
constexpr int SNT = 512;              // threads per solve workgroup (8 waves, <= 256 VGPRs)
// Register-blocked 128 x 128 tiles, 32 elements per thread:
//   row phases (L_JK y_K, X_J v, M_J y): thread (rg = t / 16, cg = t % 16)
//     holds rows 4 rg + k (k < 4), columns 2 cg + 32 j + e (j < 4, e < 2):
//     the 16 lanes of a row group read 256 contiguous bytes per load;
//   column phase (L_KJ^T x_K): thread (rg = t / 32, cg = t % 32) holds rows
//     8 rg + k (k < 8), columns 2 cg + 64 j + e (j < 2, e < 2).
constexpr int RP_ROWS = 4, RP_LANES = 16;  // row phases
constexpr int CP_ROWS = 8, CP_LANES = 32;  // column phase
constexpr int XS_LD = SB + 4;              // LDS row stride of the staged X_J
constexpr int TDS = 65;               // LDS row stride of the prep's 64 x 64 tiles
enum { SC_TICKET = 2, SC_TICKET_B = 3 };  // ticket words; ctrl[SOLVE_ERR_WORD] (1) is sticky

template <typename T>
__device__ __forceinline__ bool is_sentinel(T v);
template <>
__device__ __forceinline__ bool is_sentinel<double>(double v) {
  return __double_as_longlong(v) == (long long)-1;
}
template <>
__device__ __forceinline__ bool is_sentinel<float>(float v) {
  return __float_as_int(v) == -1;
}
template <typename T>
__device__ __forceinline__ T sentinel() {
  if constexpr (sizeof(T) == 8) return __longlong_as_double(-1ll);
  else return __int_as_float(-1);
}

// Workgroup barrier for LDS hand-offs only: unlike __syncthreads() it does not
// wait for the wave's outstanding global loads (the tile prefetches stay in
// flight across it)
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// all-reduce over the 16 lanes of a row group (DPP quad perms, then xor 4, 8)
template <typename T>
__device__ __forceinline__ T lanes16_sum(T v) {
  v += dpp_t<0xb1>(v);
  v += dpp_t<0x4e>(v);
  v += __shfl_xor(v, 4);
  return v + __shfl_xor(v, 8);
}

// ---------------------------------------------------------------------------
// prep helpers: 64 x 64 fp64 tiles in LDS (stride TDS), 256 threads, the
// v_mfma_f64_16x16x4 layout of Mfma<double> (wave w: output rows 16w..16w+15)
// a 64 x 64 tile into registers (16 loads in flight per thread; f(r, c)
// coalesced along c), then into LDS as is or transposed
template <typename F>
__device__ __forceinline__ void fetch64(double (&v)[16], F f) {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int i = threadIdx.x + 256 * q;
    v[q] = f(i >> 6, i & 63);
  }
}
template <bool TR>
__device__ __forceinline__ void put64(double* dst, const double (&v)[16]) {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int i = threadIdx.x + 256 * q;
    if (TR) dst[(i & 63) * TDS + (i >> 6)] = v[q];
    else dst[(i >> 6) * TDS + (i & 63)] = v[q];
  }
}
// acc[n] += op(A)[16w.., :] B[:, 16n..], op(A) = A or A^T
template <bool TA>
__device__ __forceinline__ void mm64(double4_t (&acc)[4], const double* A, const double* B) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int arow = 16 * wave + (lane & 15);
#pragma unroll 4
  for (int s = 0; s < 16; ++s) {
    const int k = 4 * s + (lane >> 4);
    const double a = TA ? A[k * TDS + arow] : A[arow * TDS + k];
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[n] = mfma_f64_16x16x4(a, B[k * TDS + 16 * n + (lane & 15)], acc[n]);
  }
}
__device__ __forceinline__ void zero4(double4_t (&acc)[4]) {
#pragma unroll
  for (int n = 0; n < 4; ++n) acc[n] = (double4_t){0.0, 0.0, 0.0, 0.0};
}
__device__ __forceinline__ void put4(double* dst, const double4_t (&acc)[4], double sgn) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      dst[(16 * wave + Mfma<double>::row(lane, g)) * TDS + 16 * n + (lane & 15)] = sgn * acc[n][g];
}
// acc -> 128 x 128 row-major output, quadrant (r0, c0); rows >= rmax zeroed
template <typename T>
__device__ __forceinline__ void out4(T* dst, int r0, int c0, const double4_t (&acc)[4], int rmax) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int r = r0 + 16 * wave + Mfma<double>::row(lane, g);
      dst[r * SB + c0 + 16 * n + (lane & 15)] = r < rmax ? (T)acc[n][g] : T(0);
    }
}
}  // namespace

// Five workgroups per 128-row block J (blockIdx.y = part): each builds
// X_J from the two 64 x 64 inverses (X = [[Xa, 0], [-Xb L_ba Xa, Xb]]);
// part 0 stores X_J and X_J^T, parts 1-2 the column halves of M_J, parts 3-4
// those of Q_J (fp64 MFMA, stored as T).  A part's two L operands are loaded
// with the X operands.  Rows / columns past N are zero.
template <typename T>
__global__ __launch_bounds__(256) void solve_prep_kernel(const T* __restrict__ K, int64_t ld, int N,
                                                         const T* __restrict__ Linv, T* __restrict__ X,
                                                         T* __restrict__ XT, T* __restrict__ M, T* __restrict__ Q,
                                                         int nb) {
  __shared__ double S[4][64 * TDS];  // 133 KB: Xa, Xb, X21, one L operand
  const int J = blockIdx.x, part = blockIdx.y, J0 = J * SB;
  if ((part == 1 || part == 2) && J == 0) return;
  if (part >= 3 && J + 1 >= nb) return;
  const int h = (part - 1) & 1;
  const int R = N - J0 < SB ? N - J0 : SB;
  const bool two = R > 64;
  double* Xa = S[0];
  double* Xb = S[1];
  double* X21 = S[2];
  double* Ls = S[3];
  auto Kat = [&](int r, int c) -> double { return (r < N && c < N) ? (double)K[(int64_t)r * ld + c] : 0.0; };
  const int64_t lb = (int64_t)2 * J * 64 * 64;  // Linv block of rows J0 .. J0+63
  double v0[16], v1[16], v2[16], va[16], vb[16];
  fetch64(v0, [&](int r, int c) { return (double)Linv[lb + r * 64 + c]; });
  fetch64(v1, [&](int r, int c) { return two ? (double)Linv[lb + 4096 + r * 64 + c] : 0.0; });
  fetch64(v2, [&](int r, int c) { return two ? Kat(J0 + 64 + r, J0 + c) : 0.0; });  // L_ba
  if (part == 1 || part == 2) {  // L_{J,J-1}, column half h: rows a, rows b
    const int C0 = J0 - SB + 64 * h;
    fetch64(va, [&](int r, int c) { return Kat(J0 + r, C0 + c); });
    fetch64(vb, [&](int r, int c) { return Kat(J0 + 64 + r, C0 + c); });
  } else if (part >= 3) {  // L_{J+1,J}, row half h: columns a, columns b (transposed into LDS)
    const int RR = J0 + SB + 64 * h;
    fetch64(va, [&](int r, int c) { return Kat(RR + r, J0 + c); });
    fetch64(vb, [&](int r, int c) { return Kat(RR + r, J0 + 64 + c); });
  }
  put64<false>(Xa, v0);
  put64<false>(Xb, v1);
  put64<false>(Ls, v2);
  __syncthreads();
  double4_t acc[4], bot[4];
  zero4(acc);
  mm64<false>(acc, Ls, Xa);  // L_ba Xa
  __syncthreads();
  put4(Ls, acc, 1.0);
  __syncthreads();
  zero4(acc);
  mm64<false>(acc, Xb, Ls);  // X21 = -Xb (L_ba Xa)
  put4(X21, acc, -1.0);
  __syncthreads();
  if (part == 0) {
    T* Xo = X + (int64_t)J * SB * SB;
    T* XTo = XT + (int64_t)J * SB * SB;
    for (int i = threadIdx.x; i < SB * SB; i += 256) {
      const int r = i >> 7, c = i & 127;
      double v = 0.0;
      if (r < R && c < R) v = r < 64 ? (c < 64 ? Xa[r * TDS + c] : 0.0)
                                     : (c < 64 ? X21[(r - 64) * TDS + c] : Xb[(r - 64) * TDS + c - 64]);
      Xo[r * SB + c] = (T)v;
      XTo[c * SB + r] = (T)v;
    }
    return;
  }
  zero4(acc);
  zero4(bot);
  if (part <= 2) {  // M_J = X_J L_{J,J-1}, column half h
    T* Mo = M + (int64_t)J * SB * SB;
    put64<false>(Ls, va);  // L_a,h
    __syncthreads();
    mm64<false>(acc, Xa, Ls);
    mm64<false>(bot, X21, Ls);
    __syncthreads();
    put64<false>(Ls, vb);  // L_b,h
    __syncthreads();
    mm64<false>(bot, Xb, Ls);
    out4(Mo, 0, 64 * h, acc, R);
    out4(Mo, 64, 64 * h, bot, R);
  } else {  // Q_J = X_J^T L_{J+1,J}^T, column half h (= row half of block J+1)
    T* Qo = Q + (int64_t)J * SB * SB;
    put64<true>(Ls, va);  // (L_{h,a})^T
    __syncthreads();
    mm64<true>(acc, Xa, Ls);
    __syncthreads();
    put64<true>(Ls, vb);  // (L_{h,b})^T
    __syncthreads();
    mm64<true>(acc, X21, Ls);
    mm64<true>(bot, Xb, Ls);
    out4(Qo, 0, 64 * h, acc, R);
    out4(Qo, 64, 64 * h, bot, R);
  }
}

// ---------------------------------------------------------------------------
template <typename T, bool BWD>
__global__ __launch_bounds__(SNT) void trsv128_kernel(const T* __restrict__ K, int64_t ld, int N,
                                                      const T* __restrict__ D, const T* __restrict__ X,
                                                      const T* __restrict__ XT, const T* __restrict__ M,
                                                      const T* __restrict__ Q, T* b, T* ybuf, T* xbuf,
                                                      unsigned* ctrl, int nb, const unsigned* __restrict__ skip,
                                                      int inject) {
  typedef typename Mfma<T>::vec2_t V2;
  typedef T Tile[RP_ROWS * 8];  // 32 elements: [k][j][e] (row phases) / [k][j][e] (column phase, k < 8, j < 2)
  if (skip && *skip) return;    // mixed-precision refinement already converged
  __shared__ T vs[2][SB];       // staged block vectors (bulk), then the critical vector
  __shared__ T red[SB / CP_ROWS][SB];
  __shared__ T vec[SB], bj[SB];
  // X_J (forward) / X_J^T (backward), staged at the start of the ticket so
  // the row phase after the bulk reads LDS, not HBM (stride padded: the 4 row
  // groups of a wave hit different banks)
  __shared__ __attribute__((aligned(16))) T xs[SB * XS_LD];
  __shared__ unsigned sh_ticket, sh_stop, sh_nr[2];
  unsigned* err = ctrl + SOLVE_ERR_WORD;
  const int tid = threadIdx.x;
  const int rg = tid / RP_LANES, cg = tid % RP_LANES;  // row phases
  if (tid == 0) sh_nr[0] = sh_nr[1] = 0u;

  // uniform: stage block vectors kb0, kb0 + dir (nk <= 2 of them, cnt(kb)
  // valid entries each) into vs, polled until all are complete (no sentinel
  // left); false: gave up -- after SPIN_TICKS, or when another workgroup
  // raised err (read every 32nd round, so a poll round is one load latency)
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  auto stage = [&](const T* buf, int kb0, int nk, int dir) -> bool {
    for (unsigned it = 1;; ++it) {
      lds_sync();  // earlier reads of vs / sh_nr / sh_stop are done
      const int bsel = tid / SB, e = tid % SB;
      if (tid == 0) sh_nr[(it + 1) & 1] = 0u;  // the next round's flag
      if (bsel < nk) {
        const int kb = kb0 + dir * bsel;
        const int cnt = N - kb * SB < SB ? N - kb * SB : SB;
        const T v = e < cnt ? ld_sc1(&buf[(int64_t)kb * SB + e]) : T(0);
        if (e < cnt && is_sentinel(v)) sh_nr[it & 1] = 1u;
        vs[bsel][e] = v;
      }
      if (tid == 0)
        sh_stop = __builtin_amdgcn_s_memrealtime() - t_start > SPIN_TICKS || ((it & 31u) == 0u && ld_sc1(err) != 0u);
      lds_sync();
      if (!sh_nr[it & 1]) return true;
      if (sh_stop) {
        if (tid == 0) st_sc1(err, 1u);
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  };
  // row phases: a 128 x 128 row-major tile (row stride SB) at p into t
  // (one base address per thread, immediate offsets)
  auto load_rows = [&](Tile& t, const T* p) {
    const T* q = p + RP_ROWS * rg * SB + 2 * cg;
#pragma unroll
    for (int k = 0; k < RP_ROWS; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const V2 v2 = *reinterpret_cast<const V2*>(q + k * SB + 32 * j);
        t[8 * k + 2 * j] = v2.x;
        t[8 * k + 2 * j + 1] = v2.y;
      }
  };
  auto put_xs = [&](const Tile& t) {
#pragma unroll
    for (int k = 0; k < RP_ROWS; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *reinterpret_cast<V2*>(&xs[(RP_ROWS * rg + k) * XS_LD + 2 * cg + 32 * j]) = V2{t[8 * k + 2 * j], t[8 * k + 2 * j + 1]};
  };
  // acc[k] += xs[row k, :] . v[columns of this thread]
  auto dot_xs = [&](T (&acc)[RP_ROWS], const T* v) {
    T vv[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const V2 v2 = *reinterpret_cast<const V2*>(v + 2 * cg + 32 * j);
      vv[2 * j] = v2.x;
      vv[2 * j + 1] = v2.y;
    }
#pragma unroll
    for (int k = 0; k < RP_ROWS; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const V2 x2 = *reinterpret_cast<const V2*>(&xs[(RP_ROWS * rg + k) * XS_LD + 2 * cg + 32 * j]);
        acc[k] = fma(x2.x, vv[2 * j], acc[k]);
        acc[k] = fma(x2.y, vv[2 * j + 1], acc[k]);
      }
  };
  // acc[k] += t[k, :] . v[columns of this thread]
  auto dot_rows = [&](T (&acc)[RP_ROWS], const Tile& t, const T* v) {
    T vv[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const V2 v2 = *reinterpret_cast<const V2*>(v + 2 * cg + 32 * j);
      vv[2 * j] = v2.x;
      vv[2 * j + 1] = v2.y;
    }
#pragma unroll
    for (int k = 0; k < RP_ROWS; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[k] = fma(t[8 * k + i], vv[i], acc[k]);
  };

  for (;;) {
    lds_sync();
    if (tid == 0) sh_ticket = atomicAdd(&ctrl[BWD ? SC_TICKET_B : SC_TICKET], 1u);
    lds_sync();
    const int ticket = (int)sh_ticket;
    if (ticket >= nb) return;
    // the other sweep's ticket counter, for the next launch of that sweep
    // (the previous one has completed: stream order)
    if (ticket == 0 && tid == 0) st_sc1(&ctrl[BWD ? SC_TICKET : SC_TICKET_B], 0u);

    if constexpr (!BWD) {
      // ============================================================ forward
      const int J = ticket, J0 = J * SB;
      const int R = N - J0 < SB ? N - J0 : SB;
      SSTAMP(J, 0);
      if (tid < R) st_sc1(&xbuf[J0 + tid], sentinel<T>());  // for this solve's backward launch
      // rows past N read row J0 (finite data): their sums are never used
      const T* Lrow = K + (int64_t)J0 * ld;
      const int64_t ldr = ld;
      auto row_ok = [&](int k) { return RP_ROWS * rg + k < R; };
      T acc[RP_ROWS] = {T(0), T(0), T(0), T(0)};
      Tile ta, tb;  // the next two tiles in flight
      // X_J and b_J -> LDS up front
      load_rows(ta, X + (int64_t)J * SB * SB);
      if (tid < SB) bj[tid] = tid < R ? b[J0 + tid] : T(0);
      put_xs(ta);
      auto load_tile = [&](Tile& t, int Kb) {
#pragma unroll
        for (int k = 0; k < RP_ROWS; ++k)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int64_t row = row_ok(k) ? RP_ROWS * rg + k : 0;
            const V2 v2 = *reinterpret_cast<const V2*>(Lrow + row * ldr + (int64_t)Kb * SB + 2 * cg + 32 * j);
            t[8 * k + 2 * j] = v2.x;
            t[8 * k + 2 * j + 1] = v2.y;
          }
      };
      // bulk: K < J-1.  Tiles K < J-2 in pairs as their vectors complete, the
      // next pair in flight; the last one, L_{J,J-2}, alone, so that M_J is
      // loaded into the other register tile as soon as y_{J-3} has been
      // consumed -- two hops before the hand-off needs it (loaded after the
      // bulk, its reload sat on the chain: DESIGN.md §4, the solve)
      const int Kp = J - 2;  // pairs region [0, Kp)
      const T* Mj = M + (int64_t)J * SB * SB;
      if (Kp > 0) {
        load_tile(ta, 0);
        if (Kp > 1) load_tile(tb, 1);
        else load_rows(tb, Mj);
      } else if (J >= 1) {
        if (J == 2) load_tile(ta, 0);
        load_rows(tb, Mj);
      }
      for (int Kc = 0; Kc < Kp; Kc += 2) {
        const bool two = Kc + 1 < Kp;
        if (!stage(ybuf, Kc, two ? 2 : 1, 1)) return;
        dot_rows(acc, ta, vs[0]);
        if (two) dot_rows(acc, tb, vs[1]);
        load_tile(ta, Kc + 2 < Kp ? Kc + 2 : J - 2);
        if (two) {  // tb consumed: the next pair's second tile, or M_J
          if (Kc + 3 < Kp) load_tile(tb, Kc + 3);
          else load_rows(tb, Mj);
        }
      }
      if (J >= 2) {  // L_{J,J-2} y_{J-2}
        if (!stage(ybuf, J - 2, 1, 1)) return;
        dot_rows(acc, ta, vs[0]);
      }
      SSTAMP(J, 1);
#pragma unroll
      for (int k = 0; k < RP_ROWS; ++k) acc[k] = lanes16_sum(acc[k]);
      lds_sync();  // vec / vs reuse; xs, bj staged
      if (cg == 0) {
#pragma unroll
        for (int k = 0; k < RP_ROWS; ++k) {
          const int rr = RP_ROWS * rg + k;
          vec[rr] = bj[rr] - acc[k];  // v = b_J - sum_{K<J-1} L_JK y_K
        }
      }
      lds_sync();
      T y[RP_ROWS] = {T(0), T(0), T(0), T(0)};
      dot_xs(y, vec);  // X_J v
      if (J > 0) {     // the hand-off: y_J = X_J v - M_J y_{J-1}
        SSTAMP(J, 2);
        if (!stage(ybuf, J - 1, 1, 1)) return;
        SSTAMP(J, 4);
        T d[RP_ROWS] = {T(0), T(0), T(0), T(0)};
        dot_rows(d, tb, vs[0]);
#pragma unroll
        for (int k = 0; k < RP_ROWS; ++k) y[k] -= d[k];
      }
      // inject (tests only): block 0 never publishes -> every consumer times out
#pragma unroll
      for (int k = 0; k < RP_ROWS; ++k) {
        const T yk = lanes16_sum(y[k]);
        const int rr = RP_ROWS * rg + k;
        if (cg == 0 && rr < R && !(inject && J == 0)) st_sc1(&ybuf[J0 + rr], yk);
      }
      SSTAMP(J, 3);
    } else {
      // =========================================================== backward
      const int J = nb - 1 - ticket, J0 = J * SB;
      const int R = N - J0 < SB ? N - J0 : SB;
      const bool last = J + 1 >= nb;
      // bulk: column phase; columns past the block's R give sums that are
      // never used; rows past N (ragged last block) are not read and meet
      // zero vector entries
      const int crg = tid / CP_LANES, ccg = tid % CP_LANES;
      const bool ragged = N % SB != 0;
      T acc[4] = {T(0), T(0), T(0), T(0)};  // columns 2 ccg + 64 j + e
      Tile ta, tb;
      // X_J^T and z_J = y_J / D_J -> LDS up front (y_J from the forward
      // launch: complete)
      load_rows(ta, XT + (int64_t)J * SB * SB);
      if (tid < SB) bj[tid] = tid < R ? ybuf[J0 + tid] / D[J0 + tid] : T(0);
      if (tid < R) st_sc1(&ybuf[J0 + tid], sentinel<T>());  // only this block reads y_J: reset for the next solve
      put_xs(ta);
      auto load_tile = [&](Tile& t, int Kb) {
        const int R0 = Kb * SB + CP_ROWS * crg;
        const T* p = K + (int64_t)R0 * ld + J0 + 2 * ccg;
        const bool rag = ragged && Kb == nb - 1;
#pragma unroll
        for (int k = 0; k < CP_ROWS; ++k)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const bool in = !rag || R0 + k < N;
            const V2 v2 = in ? *reinterpret_cast<const V2*>(p + (int64_t)k * ld + 64 * j) : V2{T(0), T(0)};
            t[4 * k + 2 * j] = v2.x;
            t[4 * k + 2 * j + 1] = v2.y;
          }
      };
      auto dot_cols = [&](const Tile& t, const T* v) {
        T xv[CP_ROWS];
#pragma unroll
        for (int k = 0; k < CP_ROWS; k += 2) {
          const V2 v2 = *reinterpret_cast<const V2*>(v + CP_ROWS * crg + k);
          xv[k] = v2.x;
          xv[k + 1] = v2.y;
        }
#pragma unroll
        for (int k = 0; k < CP_ROWS; ++k)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i] = fma(t[4 * k + i], xv[k], acc[i]);
      };
      // bulk: K > J+1 from the bottom.  Tiles K > J+2 in pairs as their
      // vectors complete; the last one, block J+2, alone, so that Q_J is
      // loaded into the other register tile as soon as x_{J+3} has been
      // consumed (the forward sweep's M_J schedule, mirrored)
      const int Klo = J + 3;  // pairs region [Klo, nb)
      const T* Qj = Q + (int64_t)J * SB * SB;
      if (nb - 1 >= Klo) {
        load_tile(ta, nb - 1);
        if (nb - 2 >= Klo) load_tile(tb, nb - 2);
        else load_rows(tb, Qj);
      } else if (!last) {
        if (J + 2 <= nb - 1) load_tile(ta, J + 2);
        load_rows(tb, Qj);
      }
      for (int Kc = nb - 1; Kc >= Klo; Kc -= 2) {
        const bool two = Kc - 1 >= Klo;
        if (!stage(xbuf, Kc, two ? 2 : 1, -1)) return;
        dot_cols(ta, vs[0]);
        if (two) dot_cols(tb, vs[1]);
        load_tile(ta, Kc - 2 >= Klo ? Kc - 2 : J + 2);
        if (two) {  // tb consumed: the next pair's second tile, or Q_J
          if (Kc - 3 >= Klo) load_tile(tb, Kc - 3);
          else load_rows(tb, Qj);
        }
      }
      if (J + 2 <= nb - 1) {  // L_{J+2,J}^T x_{J+2}
        if (!stage(xbuf, J + 2, 1, 1)) return;
        dot_cols(ta, vs[0]);
      }
      lds_sync();
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        red[crg][2 * ccg + 64 * j] = acc[2 * j];
        red[crg][2 * ccg + 64 * j + 1] = acc[2 * j + 1];
      }
      lds_sync();
      if (tid < SB) {
        T t = T(0);
#pragma unroll
        for (int k = 0; k < SB / CP_ROWS; ++k) t += red[k][tid];
        vec[tid] = bj[tid] - t;  // u = z_J - sum L_KJ^T x_K (zero past R)
      }
      lds_sync();
      T x[RP_ROWS] = {T(0), T(0), T(0), T(0)};
      dot_xs(x, vec);  // X_J^T u
      if (!last) {     // the hand-off: x_J = X_J^T u - Q_J x_{J+1}
        if (!stage(xbuf, J + 1, 1, 1)) return;
        T d[RP_ROWS] = {T(0), T(0), T(0), T(0)};
        dot_rows(d, tb, vs[0]);
#pragma unroll
        for (int k = 0; k < RP_ROWS; ++k) x[k] -= d[k];
      }
#pragma unroll
      for (int k = 0; k < RP_ROWS; ++k) {
        const T xk = lanes16_sum(x[k]);
        const int rr = RP_ROWS * rg + k;
        if (cg == 0 && rr < R) {
          st_sc1(&xbuf[J0 + rr], xk);
          b[J0 + rr] = xk;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
int64_t solve_prep_elems(int N) {
  const int64_t nb = (N + SB - 1) / SB;
  return 4 * nb * SB * SB;
}

template <typename T>
static hipError_t solve_prep_t(const T* K, int64_t ld, int N, const T* Linv, T* P, hipStream_t st) {
  if (N <= 0) return hipSuccess;
  const int nb = (N + SB - 1) / SB;
  const int64_t q = (int64_t)nb * SB * SB;
  hipLaunchKernelGGL(solve_prep_kernel<T>, dim3(nb, 5), dim3(256), 0, st, K, ld, N, Linv, P, P + q, P + 2 * q,
                     P + 3 * q, nb);
  return hipGetLastError();
}
hipError_t solve_stamps(unsigned long long* out) {  // DEBUG
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sstamp), sizeof(unsigned long long) * 2 * 256 * 6);
}
hipError_t solve_prep(const double* K, int64_t ld, int N, const double* Linv, double* P, hipStream_t st) {
  return solve_prep_t<double>(K, ld, N, Linv, P, st);
}
hipError_t solve_prep(const float* K, int64_t ld, int N, const float* Linv, float* P, hipStream_t st) {
  return solve_prep_t<float>(K, ld, N, Linv, P, st);
}

template <typename T>
static hipError_t solve_persistent_t(const T* K, int64_t ld, int N, const T* D, const T* P, T* b, T* ybuf, T* xbuf,
                                     unsigned* ctrl, hipStream_t st, const unsigned* skip) {
  if (N <= 0) return hipSuccess;
  if (ld % 2) return hipErrorInvalidValue;  // 2-element vector loads of the tiles
  const int nb = (N + SB - 1) / SB;
  const int64_t q = (int64_t)nb * SB * SB;
  // no per-solve memsets: each launch leaves the state the next one needs
  // (the forward resets x and the backward ticket, the backward resets y and
  // the forward ticket); solve_reset establishes it after a factorization
  hipError_t e = hipSuccess;
  // the two sweeps as two launches (each its own register allocation);
  // resident grids: one workgroup per CU
  const int grid = nb < 256 ? nb : 256;
  const int inject = debug_inject_mask() & IPMZ_INJECT_SOLVE;
  hipLaunchKernelGGL((trsv128_kernel<T, false>), dim3(grid), dim3(SNT), 0, st, K, ld, N, D, P, P + q, P + 2 * q,
                     P + 3 * q, b, ybuf, xbuf, ctrl, nb, skip, inject);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL((trsv128_kernel<T, true>), dim3(grid), dim3(SNT), 0, st, K, ld, N, D, P, P + q, P + 2 * q,
                     P + 3 * q, b, ybuf, xbuf, ctrl, nb, skip, inject);
  return hipGetLastError();
}

// one sweep of the persistent solve (forward: y = L^{-1} b into ybuf;
// backward: b = L^{-T} (ybuf / D)) -- the Bunch-Kaufman solve applies its
// block-diagonal D between the two (bk_fast_dsolve on ybuf, D = ones here)
hipError_t ldlt_solve_persistent_sweep(const double* K, int64_t ld, int N, const double* D, const double* P,
                                       double* b, double* ybuf, double* xbuf, unsigned* ctrl, bool backward,
                                       hipStream_t st, const unsigned* skip) {
  if (N <= 0) return hipSuccess;
  if (ld % 2) return hipErrorInvalidValue;
  const int nb = (N + SB - 1) / SB;
  const int64_t q = (int64_t)nb * SB * SB;
  const int grid = nb < 256 ? nb : 256;
  const int inject = debug_inject_mask() & IPMZ_INJECT_SOLVE;
  if (backward)
    hipLaunchKernelGGL((trsv128_kernel<double, true>), dim3(grid), dim3(SNT), 0, st, K, ld, N, D, P, P + q, P + 2 * q,
                       P + 3 * q, b, ybuf, xbuf, ctrl, nb, skip, inject);
  else
    hipLaunchKernelGGL((trsv128_kernel<double, false>), dim3(grid), dim3(SNT), 0, st, K, ld, N, D, P, P + q,
                       P + 2 * q, P + 3 * q, b, ybuf, xbuf, ctrl, nb, skip, inject);
  return hipGetLastError();
}

namespace {
// up to 6 word ranges, each filled with its own value: one launch for what
// would be one memset (and one launch gap) each
struct FillJob {
  unsigned* p[6];
  int64_t n[6];
  unsigned v[6];
};
__global__ __launch_bounds__(256) void fill_words_kernel(FillJob f) {
  const int r = blockIdx.y;
  unsigned* const p = f.p[r];
  const unsigned v = f.v[r];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < f.n[r]; i += (int64_t)gridDim.x * 256) p[i] = v;
}
}  // namespace

hipError_t solve_reset(void* ybuf, void* xbuf, size_t elem, int N, unsigned* ctrl, hipStream_t st, int* info,
                       unsigned* words, int64_t nwords, int* info2) {
  FillJob f{};
  int cnt = 0;
  int64_t most = 0;
  auto add = [&](void* p, int64_t n, unsigned v) {
    if (!p || n <= 0) return;
    f.p[cnt] = static_cast<unsigned*>(p);
    f.n[cnt] = n;
    f.v[cnt++] = v;
    most = n > most ? n : most;
  };
  add(ctrl, IPMZ_SOLVE_CTRL_WORDS, 0u);  // tickets + sticky error
  add(ybuf, (int64_t)N * (int64_t)elem / 4, ~0u);
  add(xbuf, (int64_t)N * (int64_t)elem / 4, ~0u);
  add(info, 1, 0x7f7f7f7fu);  // "no pivot failed" (the byte pattern of hipMemset 0x7f)
  add(info2, 1, 0x7f7f7f7fu);
  add(words, nwords, 0u);
  if (!cnt) return hipSuccess;
  const int64_t gx = (most + 255) / 256;
  hipLaunchKernelGGL(fill_words_kernel, dim3((unsigned)(gx < 64 ? gx : 64), cnt), dim3(256), 0, st, f);
  return hipGetLastError();
}

hipError_t ldlt_solve_persistent(const double* K, int64_t ld, int N, const double* D, const double* P, double* b,
                                 double* ybuf, double* xbuf, unsigned* ctrl, hipStream_t st) {
  return solve_persistent_t<double>(K, ld, N, D, P, b, ybuf, xbuf, ctrl, st, nullptr);
}
hipError_t ldlt_solve_persistent(const float* K, int64_t ld, int N, const float* D, const float* P, float* b,
                                 float* ybuf, float* xbuf, unsigned* ctrl, hipStream_t st, const unsigned* skip) {
  return solve_persistent_t<float>(K, ld, N, D, P, b, ybuf, xbuf, ctrl, st, skip);
}

}  // namespace ipmz
