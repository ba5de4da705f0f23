// Single-launch triangular solve with the LDL^T factor, x = L^{-T} D^{-1} L^{-1} b
// (LinearSolvers::overwriting_solve_ldlt, LinearSolvers.cpp:44-74), organised
// around ONE chain workgroup that owns the whole dependency chain.
//
// The dequeued solve (trsv_persist.hip) hands every 64-row block from one
// workgroup to the next through memory: on MI355X that is a cross-XCD round
// trip or two per block (~2.4 us), 2 x 176 of them per C3 solve.  Here:
//   ticket 0        : the CHAIN.  Forward, block J = 0 .. nblk-1:
//                       v = b_J - s_J - L[J, J-1] y_{J-1} - L[J, J-2] y_{J-2}
//                       y_J = Linv_J v
//                     with y_{J-1}, y_{J-2} from its own LDS ring (no memory
//                     round trip), s_J from a helper.  Then backward,
//                     J = nblk-1 .. 0:
//                       u = y_J / D_J - t_J - L[J+1, J]^T x_{J+1} - L[J+2, J]^T x_{J+2}
//                       x_J = Linv_J^T u
//   other tickets   : HELPERS, one per block: s_J = sum_{K <= J-3} L[J, K] y_K
//                     (forward) and t_J = sum_{K >= J+3} L[K, J]^T x_K
//                     (backward), polling y / x as they appear.  A helper's
//                     last input is three chain steps old when the chain needs
//                     its result, so the chain rarely waits.
// Hand-off (no flags): y, x, s, t start as an all-ones bit pattern (a NaN
// payload arithmetic never produces) and are stored with agent-scope (sc1)
// atomic stores, one aligned 8-byte element each; a consumer polls each
// element with agent-scope loads until it is not the sentinel.  Helpers
// only wait on the chain (ticket 0, always running: tickets are taken by
// running workgroups in order) and the chain on helpers that running
// workgroups will reach, so the grid cannot deadlock.  Every spin is bounded
// (SPIN_TICKS) and raises an error word.  The chain's L tiles, L^{-1} rows
// and rhs are loaded one step ahead.
// Summation order is fixed: the result is deterministic.
#include "common.h"
#include "kernels.h"
#include "sync.h"

#include <type_traits>

namespace ipmz {

namespace {
constexpr int CNT = 512;  // threads per workgroup: 8 doubles of a 64 x 64 tile each
constexpr int CW = CNT / 64;  // waves
constexpr int NB = 64;

__device__ __forceinline__ bool is_sent(double v) { return __double_as_longlong(v) == (long long)-1; }
// all-reduce over aligned groups of 8 lanes (quad xor 1, xor 2, then the
// row_half_mirror partner in the other quad)
__device__ __forceinline__ double oct_sum(double v) {
  v += dpp_t<0xb1>(v);
  v += dpp_t<0x4e>(v);
  v += dpp_t<0x141>(v);
  return v;
}
// poll src[i] (i < count) until it is not the sentinel; bounded
__device__ __forceinline__ bool poll1(const double* src, double& v, unsigned* err) {
  v = ld_sc1(src);
  if (!is_sent(v)) return true;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (is_sent(v)) {
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS ||
        __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    v = ld_sc1(src);
  }
  return true;
}
__device__ __forceinline__ bool all_ok(bool ok, unsigned* sh) {
  if (threadIdx.x == 0) *sh = 1u;
  __syncthreads();
  if (!ok) *sh = 0u;
  __syncthreads();
  return *sh != 0u;
}

// row-wise 64 x 64 tile piece of thread t: row r = t >> 3, columns c0 .. c0+7
struct RowTile {
  double v[8];
  __device__ __forceinline__ void load(const double* K, int64_t ld, int row, int col, bool in) {
    const double* p = K + (int64_t)(in ? row : 0) * ld + col;
#pragma unroll
    for (int q = 0; q < 8; q += 2) {
      const double2 d2 = *reinterpret_cast<const double2*>(p + q);
      v[q] = in ? d2.x : 0.0;
      v[q + 1] = in ? d2.y : 0.0;
    }
  }
};
// column-wise piece: rows R0 + q (q < 8), column col
struct ColTile {
  double v[8];
  // rows past N read row N-1 (finite; their x multipliers are zero); no
  // per-element branches
  __device__ __forceinline__ void load(const double* K, int64_t ld, int N, int R0, int col) {
    const double* p = K + col;
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = p[(int64_t)(R0 + q < N ? R0 + q : N - 1) * ld];
  }
};
}  // namespace

__device__ __forceinline__ int rows_of(int N, int J) { return N - J * NB < NB ? N - J * NB : NB; }

// forward chain registers of one block J
struct FwdSet {
  RowTile a1, a2;
  double li[8], bv, sj;
  __device__ __forceinline__ void fetch(const double* K, int64_t ld, const double* Linv, const double* b, int nblk,
                                        int N, int J, int r, int c0) {
    if (J >= nblk) return;
    const int J0 = J * NB;
    const bool in = r < rows_of(N, J);
    if (J >= 1) a1.load(K, ld, J0 + r, (J - 1) * NB + c0, in);
    if (J >= 2) a2.load(K, ld, J0 + r, (J - 2) * NB + c0, in);
    const double* lp = Linv + (int64_t)J * NB * NB + r * NB + c0;
#pragma unroll
    for (int q = 0; q < 8; q += 2) {
      const double2 d2 = *reinterpret_cast<const double2*>(lp + q);
      li[q] = d2.x;
      li[q + 1] = d2.y;
    }
    bv = in ? b[J0 + r] : 0.0;
    // the helper's partial s_J, one step early (re-polled if not there yet)
    sj = (J >= 3 && (threadIdx.x & 7) == 0 && in) ? ld_sc1(&sbuf[J0 + r]) : 0.0;
  }
  const double* sbuf = nullptr;
};
// backward chain registers of one block J
struct BwdSet {
  ColTile t1, t2;
  double lt[8], zv, tj;
  const double* tbuf = nullptr;
  __device__ __forceinline__ void fetch(const double* K, int64_t ld, const double* Linv, const double* D,
                                        const double* ybuf, int nblk, int N, int J, int cc, int rq) {
    if (J < 0) return;
    const int J0 = J * NB;
    const bool in = cc < rows_of(N, J);
    if (J + 1 < nblk) t1.load(K, ld, N, (J + 1) * NB + rq, J0 + cc);  // (J < nblk-1: a full block)
    if (J + 2 < nblk) t2.load(K, ld, N, (J + 2) * NB + rq, J0 + cc);
#pragma unroll
    for (int q = 0; q < 8; ++q) lt[q] = Linv[(int64_t)J * NB * NB + (rq + q) * NB + cc];
    const int e = in ? J0 + cc : J0;
    zv = ld_sc1(&ybuf[e]) / D[e];  // z_J = y_J / D_J (lanes past N: unused)
    tj = (J + 3 < nblk && threadIdx.x < NB && in) ? ld_sc1(&tbuf[J0 + cc]) : 0.0;  // helper partial, early
  }
};

// v = b_J - s_J - L[J, J-1] y_{J-1} - L[J, J-2] y_{J-2};  y_J = Linv_J v
__device__ __forceinline__ bool fwd_step(const FwdSet& S, int J, int N, double (*ring)[NB], double* vec,
                                         double* ybuf, const double* sbuf, unsigned* err, unsigned* sh_ok, int r,
                                         int c0) {
  const int J0 = J * NB, rows = rows_of(N, J);
  const int tid = threadIdx.x;
  double acc = 0.0;
  if (J >= 1) {
    const double* y1 = ring[(J - 1) % 3];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc = fma(S.a1.v[q], y1[c0 + q], acc);
  }
  if (J >= 2) {
    const double* y2 = ring[(J - 2) % 3];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc = fma(S.a2.v[q], y2[c0 + q], acc);
  }
  acc = oct_sum(acc);
  double sj = S.sj;
  bool ok = true;
  if (J >= 3 && (tid & 7) == 0 && r < rows && is_sent(sj)) ok = poll1(&sbuf[J0 + r], sj, err);
  if (!all_ok(ok, sh_ok)) return false;
  if ((tid & 7) == 0) vec[r] = r < rows ? (S.bv - sj) - acc : 0.0;
  __syncthreads();
  double y = 0.0;
#pragma unroll
  for (int q = 0; q < 8; ++q) y = fma(S.li[q], vec[c0 + q], y);
  y = oct_sum(y);
  if ((tid & 7) == 0) {
    ring[J % 3][r] = y;
    if (r < rows) st_sc1(&ybuf[J0 + r], y);
  }
  __syncthreads();
  return true;
}

__device__ __forceinline__ double wsum(const double (*red)[NB], int c);
// u = z_J - t_J - L[J+1, J]^T x_{J+1} - L[J+2, J]^T x_{J+2};  x_J = Linv_J^T u
__device__ __forceinline__ bool bwd_step(const BwdSet& S, int J, int nblk, int N, double (*ring)[NB], double* vec,
                                         double (*red)[NB], double* b, double* xbuf, const double* tbuf,
                                         unsigned* err, unsigned* sh_ok, int cc, int rq) {
  const int J0 = J * NB, rows = rows_of(N, J);
  const int tid = threadIdx.x, wave = tid >> 6;
  double acc = 0.0;
  if (J + 1 < nblk) {
    const double* x1 = ring[(J + 1) % 3];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc = fma(S.t1.v[q], x1[rq + q], acc);
  }
  if (J + 2 < nblk) {
    const double* x2 = ring[(J + 2) % 3];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc = fma(S.t2.v[q], x2[rq + q], acc);
  }
  red[wave][cc] = acc;
  double tj = S.tj;
  bool ok = true;
  if (J + 3 < nblk && tid < NB && cc < rows && is_sent(tj)) ok = poll1(&tbuf[J0 + cc], tj, err);
  if (!all_ok(ok, sh_ok)) return false;  // (its barriers also publish red)
  if (tid < NB) vec[tid] = tid < rows ? (S.zv - tj) - wsum(red, tid) : 0.0;
  __syncthreads();
  double x = 0.0;
#pragma unroll
  for (int q = 0; q < 8; ++q) x = fma(S.lt[q], vec[rq + q], x);
  red[wave][cc] = x;
  __syncthreads();
  if (tid < NB) {
    const double xv = wsum(red, tid);
    ring[J % 3][tid] = tid < rows ? xv : 0.0;
    if (tid < rows) {
      st_sc1(&xbuf[J0 + tid], xv);
      b[J0 + tid] = xv;
    }
  }
  __syncthreads();
  return true;
}

__device__ __forceinline__ double wsum(const double (*red)[NB], int c) {
  double t = red[0][c];
#pragma unroll
  for (int w = 1; w < CW; ++w) t += red[w][c];
  return t;
}

__global__ __launch_bounds__(CNT) void trsv_chain_kernel(const double* __restrict__ K, int64_t ld, int N,
                                                         const double* __restrict__ D,
                                                         const double* __restrict__ Linv, double* b, double* ybuf,
                                                         double* sbuf, double* xbuf, double* tbuf, unsigned* ctrl,
                                                         int nblk) {
  __shared__ double ring[3][NB];  // chain: y / x of the last three blocks
  __shared__ double vec[8 * NB];  // helpers: polled y / x of up to 8 blocks; chain: v / u
  __shared__ double red[CW][NB];
  __shared__ unsigned sh_ticket, sh_ok;
  unsigned* counter = ctrl;
  unsigned* err = ctrl + 1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = tid >> 3, c0 = (tid & 7) * 8;  // row-wise layout
  const int cc = lane, rq = wave * 8;           // column-wise layout
  auto rows_of = [&](int J) { return ipmz::rows_of(N, J); };

  for (;;) {
    if (tid == 0) sh_ticket = atomicAdd(counter, 1u);
    __syncthreads();
    const int ticket = (int)sh_ticket;
    __syncthreads();
    const int nhf = nblk > 3 ? nblk - 3 : 0;  // forward helpers: blocks 3 .. nblk-1
    if (ticket >= 1 + 2 * nhf) return;

    if (ticket == 0) {
      // ======================================================== the chain
      // forward: tiles (J, J-1), (J, J-2), Linv_J rows and b_J of the next
      // block are loaded while this one computes (register sets A / B)
      FwdSet A, B;
      A.sbuf = B.sbuf = sbuf;
      A.fetch(K, ld, Linv, b, nblk, N, 0, r, c0);
#pragma unroll 1
      for (int J = 0; J < nblk; J += 2) {
        B.fetch(K, ld, Linv, b, nblk, N, J + 1, r, c0);
        if (!fwd_step(A, J, N, ring, vec, ybuf, sbuf, err, &sh_ok, r, c0)) return;
        if (J + 1 >= nblk) break;
        A.fetch(K, ld, Linv, b, nblk, N, J + 2, r, c0);
        if (!fwd_step(B, J + 1, N, ring, vec, ybuf, sbuf, err, &sh_ok, r, c0)) return;
      }
      // backward: tiles (J+1, J)^T, (J+2, J)^T, Linv_J^T columns and
      // z_J = y_J / D_J of the next block loaded while this one computes
      BwdSet P, Q;
      P.tbuf = Q.tbuf = tbuf;
      P.fetch(K, ld, Linv, D, ybuf, nblk, N, nblk - 1, cc, rq);
#pragma unroll 1
      for (int J = nblk - 1; J >= 0; J -= 2) {
        Q.fetch(K, ld, Linv, D, ybuf, nblk, N, J - 1, cc, rq);
        if (!bwd_step(P, J, nblk, N, ring, vec, red, b, xbuf, tbuf, err, &sh_ok, cc, rq)) return;
        if (J - 1 < 0) break;
        P.fetch(K, ld, Linv, D, ybuf, nblk, N, J - 2, cc, rq);
        if (!bwd_step(Q, J - 1, nblk, N, ring, vec, red, b, xbuf, tbuf, err, &sh_ok, cc, rq)) return;
      }
    } else if (ticket <= nhf) {
      // ================================================ forward helper
      // s_J = sum_{K = 0}^{J-3} L[J, K] y_K, y polled eight blocks at a time
      const int J = ticket + 2, J0 = J * NB, rows = rows_of(J);
      const int nk = J - 2;  // K = 0 .. J-3
      const bool in = r < rows;
      RowTile cur, nxt;
      cur.load(K, ld, J0 + r, c0, in);
      double acc = 0.0;
      for (int k0 = 0; k0 < nk; k0 += CW) {
        const int kc = nk - k0 < CW ? nk - k0 : CW;
        double yv = 0.0;
        const bool ok = tid < kc * NB ? poll1(&ybuf[k0 * NB + tid], yv, err) : true;
        vec[tid] = yv;
        if (!all_ok(ok, &sh_ok)) return;
        for (int k = 0; k < kc; ++k) {
          if (k0 + k + 1 < nk) nxt.load(K, ld, J0 + r, (k0 + k + 1) * NB + c0, in);
#pragma unroll
          for (int q = 0; q < 8; ++q) acc = fma(cur.v[q], vec[k * NB + c0 + q], acc);
#pragma unroll
          for (int q = 0; q < 8; ++q) cur.v[q] = nxt.v[q];
        }
        __syncthreads();  // vec reused
      }
      acc = oct_sum(acc);
      if ((tid & 7) == 0 && in) st_sc1(&sbuf[J0 + r], acc);
    } else {
      // =============================================== backward helper
      // t_J = sum_{K = J+3}^{nblk-1} L[K, J]^T x_K, x polled as it appears
      // (from the last block down), eight blocks at a time
      const int J = (ticket - nhf) - 1, J0 = J * NB, rows = rows_of(J);  // J = 0 .. nhf-1
      const bool in = cc < rows;
      const int kfirst = nblk - 1, klast = J + 3;  // K runs kfirst down to klast
      ColTile cur, nxt;
      cur.load(K, ld, N, kfirst * NB + rq, J0 + cc);
      double acc = 0.0;
      for (int k0 = kfirst; k0 >= klast; k0 -= CW) {
        const int kc = k0 - klast + 1 < CW ? k0 - klast + 1 : CW;  // blocks k0, k0-1, .., k0-kc+1
        const int kb = tid >> 6, e = tid & 63;
        double xv = 0.0;
        const bool ok = (kb < kc && (k0 - kb) * NB + e < N) ? poll1(&xbuf[(k0 - kb) * NB + e], xv, err) : true;
        vec[tid] = xv;
        if (!all_ok(ok, &sh_ok)) return;
        for (int k = 0; k < kc; ++k) {
          const int Kb = k0 - k;
          if (Kb - 1 >= klast) nxt.load(K, ld, N, (Kb - 1) * NB + rq, J0 + cc);
#pragma unroll
          for (int q = 0; q < 8; ++q) acc = fma(cur.v[q], vec[k * NB + rq + q], acc);
#pragma unroll
          for (int q = 0; q < 8; ++q) cur.v[q] = nxt.v[q];
        }
        __syncthreads();
      }
      red[wave][cc] = acc;
      __syncthreads();
      if (tid < NB && tid < rows)
        st_sc1(&tbuf[J0 + tid], wsum(red, tid));
      __syncthreads();
    }
  }
}

hipError_t ldlt_solve_chain(const double* K, int64_t ld, int N, const double* D, const double* Linv, double* b,
                            double* ybuf, double* sbuf, double* xbuf, double* tbuf, unsigned* ctrl, hipStream_t st) {
  if (N <= 0) return hipSuccess;
  const int nblk = (N + NB - 1) / NB;
  hipError_t e;
  if ((e = hipMemsetAsync(ctrl, 0, 2 * sizeof(unsigned), st)) != hipSuccess) return e;
  for (double* p : {ybuf, sbuf, xbuf, tbuf})
    if ((e = hipMemsetAsync(p, 0xff, (size_t)N * sizeof(double), st)) != hipSuccess) return e;
  const int tickets = 1 + 2 * (nblk > 3 ? nblk - 3 : 0);
  const int grid = tickets < 512 ? tickets : 512;
  hipLaunchKernelGGL(trsv_chain_kernel, dim3(grid), dim3(CNT), 0, st, K, ld, N, D, Linv, b, ybuf, sbuf, xbuf, tbuf,
                     ctrl, nblk);
  return hipGetLastError();
}

}  // namespace ipmz
