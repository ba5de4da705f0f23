// Single-launch, sync-free triangular solve with the LDL^T factor:
//   x = L^{-T} D^{-1} L^{-1} b   (LinearSolvers.cpp:44-74)
//
// The forward sweep (Ly = b, z = y / D) and the backward sweep (L^T x = z)
// are 2 * nblk "tickets" of NB-row blocks, claimed in dependency order from
// a device counter by whichever workgroup is running (dequeue pattern): a
// ticket only ever waits on LOWER tickets, all of which belong to running
// workgroups, so the grid cannot deadlock whatever the dispatch order.
//
//   forward block J  : v = b_J - sum_{K<J} L_JK y_K ; y_J = Linv_J v ;
//                      z_J = y_J / D_J                      -> flag F[J]
//   backward block J : u = z_J - sum_{K>J} L_KJ^T x_K ; x_J = Linv_J^T u
//                                                          -> flag B[J]
// Every off-diagonal tile is streamed into registers BEFORE the flag it
// needs is polled, so the critical path per block is one hand-off plus one
// NB x NB tile product plus the diagonal-block apply.
//
// Hand-off protocol (cdna_hip_programming.md §6 Guideline 16, "Valid forms"
// row 1): block vectors are stored write-through (sc1: relaxed agent-scope
// atomic stores), every storing wave drains vmcnt(0), a workgroup barrier,
// then ONE lane stores the flag with a relaxed agent-scope atomic; consumers
// poll the flag with relaxed agent-scope loads and read the vectors with sc1
// loads only.  Flags are zeroed by a memset node before every launch.  Spins
// are bounded: on timeout the kernel records an error word and gives up.
#include "common.h"
#include "kernels.h"
#include "sync.h"

#include <cstdlib>
#include <cstring>

namespace ipmz {

namespace {
constexpr int PNT = 256;                 // threads per workgroup

// quad (4-lane) all-reduce on the VALU
template <typename T>
__device__ __forceinline__ T quad_sum(T v) {
  v += dpp_t<0xb1>(v);
  v += dpp_t<0x4e>(v);
  return v;
}
}  // namespace

// NB = 64: forward tiles are read row-wise (thread t: row t>>2, 16 columns
// (t&3)*16..+16 -> 8 x 16-byte loads), backward tiles column-wise (thread t:
// column t&63, rows (t>>6)*16..+16).
template <typename T, int NB>
__global__ __launch_bounds__(PNT) void trsv_persistent_kernel(const T* __restrict__ K, int64_t ld, int N,
                                                              const T* __restrict__ D, const T* __restrict__ Linv,
                                                              T* b, T* ybuf, T* zbuf, unsigned* ctrl, int nblk,
                                                              const unsigned* __restrict__ skip) {
  typedef typename Mfma<T>::vec2_t V2;
  if (skip && *skip) return;  // mixed-precision refinement already converged
  static_assert(NB == 64, "persistent solve is written for 64-row blocks");
  __shared__ T vec[NB];      // y_K / x_K of the tile being applied, then v / u
  __shared__ T red[4][NB];   // cross-wave reduction (backward)
  __shared__ unsigned sh_ticket, sh_ok;
  unsigned* counter = ctrl;
  unsigned* err = ctrl + 1;
  unsigned* fflag = ctrl + 2;
  unsigned* bflag = ctrl + 2 + nblk;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;

  for (;;) {
    if (tid == 0) sh_ticket = atomicAdd(counter, 1u);
    __syncthreads();
    const int ticket = (int)sh_ticket;
    __syncthreads();
    if (ticket >= 2 * nblk) return;

    if (ticket < nblk) {
      // ------------------------------------------------------------ forward
      const int J = ticket, J0 = J * NB;
      const int rows = N - J0 < NB ? N - J0 : NB;
      const int r = tid >> 2, c0 = (tid & 3) * 16;
      // diagonal-block inverse row r (Linv_J, NB x NB) and b_J[r]
      T li[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) li[q] = Linv[(int64_t)J * NB * NB + r * NB + c0 + q];
      T acc = T(0);
      T tile[16];
      auto load_tile = [&](int Kb) {
        const bool in = r < rows;
        const T* p = K + (int64_t)(J0 + (in ? r : 0)) * ld + Kb * NB + c0;
#pragma unroll
        for (int q = 0; q < 16; q += 2) {
          const V2 v2 = *reinterpret_cast<const V2*>(p + q);
          tile[q] = in ? v2.x : T(0);
          tile[q + 1] = in ? v2.y : T(0);
        }
      };
      if (J > 0) load_tile(0);
      for (int Kb = 0; Kb < J; ++Kb) {
        if (!wait_flag(&fflag[Kb], err, &sh_ok)) return;
        if (tid < NB) vec[tid] = ld_sc1(&ybuf[Kb * NB + tid]);
        __syncthreads();
        T cur[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) cur[q] = tile[q];
        if (Kb + 1 < J) load_tile(Kb + 1);  // next tile in flight during this product
#pragma unroll
        for (int q = 0; q < 16; ++q) acc = fma(cur[q], vec[c0 + q], acc);
        __syncthreads();
      }
      acc = quad_sum(acc);
      const T bv = r < rows ? b[J0 + r] : T(0);
      if ((tid & 3) == 0) vec[r] = bv - acc;  // v = b_J - L_J,<J y
      __syncthreads();
      T y = T(0);
#pragma unroll
      for (int q = 0; q < 16; ++q) y = fma(li[q], vec[c0 + q], y);
      y = quad_sum(y);
      if ((tid & 3) == 0 && r < rows) {
        st_sc1(&ybuf[J0 + r], y);
        st_sc1(&zbuf[J0 + r], y / D[J0 + r]);
      }
      publish(&fflag[J]);
    } else {
      // ----------------------------------------------------------- backward
      const int J = nblk - 1 - (ticket - nblk), J0 = J * NB;
      const int rows = N - J0 < NB ? N - J0 : NB;
      const int c = lane, rq = wave * 16;
      // Linv_J^T column c: Linv_J[rq + q][c]
      T li[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) li[q] = Linv[(int64_t)J * NB * NB + (rq + q) * NB + c];
      T acc = T(0);
      T tile[16];
      auto load_tile = [&](int Kb) {  // L_KJ rows Kb*NB + rq.., column J0 + c
        const int R0 = Kb * NB + rq;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int row = R0 + q;
          tile[q] = (row < N && c < rows) ? K[(int64_t)row * ld + J0 + c] : T(0);
        }
      };
      if (J + 1 < nblk) load_tile(nblk - 1);
      if (!wait_flag(&fflag[J], err, &sh_ok)) return;  // z_J ready
      for (int Kb = nblk - 1; Kb > J; --Kb) {
        if (!wait_flag(&bflag[Kb], err, &sh_ok)) return;
        if (tid < NB) vec[tid] = (Kb * NB + tid < N) ? ld_sc1(&b[Kb * NB + tid]) : T(0);
        __syncthreads();
        T cur[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) cur[q] = tile[q];
        if (Kb - 1 > J) load_tile(Kb - 1);
#pragma unroll
        for (int q = 0; q < 16; ++q) acc = fma(cur[q], vec[rq + q], acc);
        __syncthreads();
      }
      red[wave][c] = acc;
      __syncthreads();
      if (tid < NB) {
        const T t = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
        vec[tid] = tid < rows ? ld_sc1(&zbuf[J0 + tid]) - t : T(0);  // u = z_J - sum L_KJ^T x_K
      }
      __syncthreads();
      T x = T(0);
#pragma unroll
      for (int q = 0; q < 16; ++q) x = fma(li[q], vec[rq + q], x);
      red[wave][c] = x;
      __syncthreads();
      if (tid < rows) st_sc1(&b[J0 + tid], (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]));
      publish(&bflag[J]);
    }
  }
}

// ---------------------------------------------------------------------------
// The same dequeued solve with the hand-off carried by the data itself: the
// block vectors y (forward) and x (backward) start as an all-ones bit
// pattern (a NaN payload arithmetic never produces) and a consumer polls its
// 64 elements with agent-scope loads until none is the sentinel.  Each
// element is one aligned 8-byte store, so seeing it is seeing its final
// value: no flag word, no producer-side drain + barrier + flag store, no
// flag -> data round trip (two cross-XCD latencies per hop become one).
// z = y / D is recomputed by the backward block from y (same rounding).
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
// wave 0 polls src[0 .. count) into dst (LDS; zeros past count); the
// workgroup leaves together.  Bounded like wait_flag.
template <typename T>
__device__ __forceinline__ bool poll_vec(const T* src, int count, T* dst, unsigned* err, unsigned* sh_ok) {
  const int lane = threadIdx.x & 63;
  if (threadIdx.x < 64) {
    bool ok = true;
    T v = T(0);
    if (lane < count) {
      v = ld_sc1(&src[lane]);
      if (is_sentinel(v)) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (is_sentinel(v)) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS ||
              __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
            ok = false;
            break;
          }
          v = ld_sc1(&src[lane]);
        }
      }
    }
    dst[lane] = v;
    const unsigned long long bad = __ballot(!ok);
    if (lane == 0) {
      *sh_ok = bad == 0ull;
      if (bad) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return *sh_ok != 0;
}

template <typename T, int NB>
__global__ __launch_bounds__(PNT) void trsv_sentinel_kernel(const T* __restrict__ K, int64_t ld, int N,
                                                            const T* __restrict__ D, const T* __restrict__ Linv,
                                                            T* b, T* ybuf, T* xbuf, unsigned* ctrl, int nblk,
                                                            const unsigned* __restrict__ skip) {
  typedef typename Mfma<T>::vec2_t V2;
  if (skip && *skip) return;  // mixed-precision refinement already converged
  static_assert(NB == 64, "persistent solve is written for 64-row blocks");
  __shared__ T vec[NB];
  __shared__ T red[4][NB];
  __shared__ unsigned sh_ticket, sh_ok;
  unsigned* counter = ctrl;
  unsigned* err = ctrl + 1;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;

  for (;;) {
    if (tid == 0) sh_ticket = atomicAdd(counter, 1u);
    __syncthreads();
    const int ticket = (int)sh_ticket;
    __syncthreads();
    if (ticket >= 2 * nblk) return;

    if (ticket < nblk) {
      // ------------------------------------------------------------ forward
      const int J = ticket, J0 = J * NB;
      const int rows = N - J0 < NB ? N - J0 : NB;
      const int r = tid >> 2, c0 = (tid & 3) * 16;
      T li[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) li[q] = Linv[(int64_t)J * NB * NB + r * NB + c0 + q];
      T acc = T(0);
      T tile[16];
      auto load_tile = [&](int Kb) {
        const bool in = r < rows;
        const T* p = K + (int64_t)(J0 + (in ? r : 0)) * ld + Kb * NB + c0;
#pragma unroll
        for (int q = 0; q < 16; q += 2) {
          const V2 v2 = *reinterpret_cast<const V2*>(p + q);
          tile[q] = in ? v2.x : T(0);
          tile[q + 1] = in ? v2.y : T(0);
        }
      };
      if (J > 0) load_tile(0);
      for (int Kb = 0; Kb < J; ++Kb) {
        if (!poll_vec(&ybuf[Kb * NB], NB, vec, err, &sh_ok)) return;
        T cur[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) cur[q] = tile[q];
        if (Kb + 1 < J) load_tile(Kb + 1);  // next tile in flight during this product
#pragma unroll
        for (int q = 0; q < 16; ++q) acc = fma(cur[q], vec[c0 + q], acc);
        __syncthreads();
      }
      acc = quad_sum(acc);
      const T bv = r < rows ? b[J0 + r] : T(0);
      if ((tid & 3) == 0) vec[r] = bv - acc;  // v = b_J - L_J,<J y
      __syncthreads();
      T y = T(0);
#pragma unroll
      for (int q = 0; q < 16; ++q) y = fma(li[q], vec[c0 + q], y);
      y = quad_sum(y);
      if ((tid & 3) == 0 && r < rows) st_sc1(&ybuf[J0 + r], y);
      __syncthreads();  // vec reused by the next ticket
    } else {
      // ----------------------------------------------------------- backward
      const int J = nblk - 1 - (ticket - nblk), J0 = J * NB;
      const int rows = N - J0 < NB ? N - J0 : NB;
      const int c = lane, rq = wave * 16;
      T li[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) li[q] = Linv[(int64_t)J * NB * NB + (rq + q) * NB + c];
      T acc = T(0);
      T tile[16];
      auto load_tile = [&](int Kb) {  // L_KJ rows Kb*NB + rq.., column J0 + c
        const int R0 = Kb * NB + rq;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int row = R0 + q;
          tile[q] = (row < N && c < rows) ? K[(int64_t)row * ld + J0 + c] : T(0);
        }
      };
      if (J + 1 < nblk) load_tile(nblk - 1);
      for (int Kb = nblk - 1; Kb > J; --Kb) {
        const int cnt = N - Kb * NB < NB ? N - Kb * NB : NB;
        if (!poll_vec(&xbuf[Kb * NB], cnt, vec, err, &sh_ok)) return;
        T cur[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) cur[q] = tile[q];
        if (Kb - 1 > J) load_tile(Kb - 1);
#pragma unroll
        for (int q = 0; q < 16; ++q) acc = fma(cur[q], vec[rq + q], acc);
        __syncthreads();
      }
      red[wave][c] = acc;
      // own y_J (-> z_J = y_J / D_J, as the forward sweep's z)
      if (!poll_vec(&ybuf[J0], rows, vec, err, &sh_ok)) return;
      if (tid < NB) {
        const T t = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
        vec[tid] = tid < rows ? vec[tid] / D[J0 + tid] - t : T(0);  // u = z_J - sum L_KJ^T x_K
      }
      __syncthreads();
      T x = T(0);
#pragma unroll
      for (int q = 0; q < 16; ++q) x = fma(li[q], vec[rq + q], x);
      red[wave][c] = x;
      __syncthreads();
      if (tid < rows) {
        const T xv = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
        st_sc1(&xbuf[J0 + tid], xv);
        b[J0 + tid] = xv;
      }
      __syncthreads();
    }
  }
}

template <typename T>
static hipError_t solve_persistent_t(const T* K, int64_t ld, int N, const T* D, const T* Linv, int nbi, T* b, T* ybuf,
                                     T* zbuf, unsigned* ctrl, hipStream_t st, const unsigned* skip = nullptr) {
  if (N <= 0) return hipSuccess;
  if (nbi != 64) return hipErrorInvalidValue;
  const int nblk = (N + 63) / 64;
  hipError_t e = hipMemsetAsync(ctrl, 0, (size_t)(2 + 2 * nblk) * sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  // resident grid: 3 workgroups per CU fit (LDS ~2.6 KB, < 128 VGPRs); the
  // dequeue makes residency a performance matter only
  int grid = 2 * nblk < 512 ? 2 * nblk : 512;
  // default: sentinel hand-off (same speed as the flag protocol at C3, one
  // fewer memory round trip per block); IPMZ_SOLVE=flags selects the flags
  static const bool flags = [] {
    const char* v = std::getenv("IPMZ_SOLVE");
    return v && !std::strcmp(v, "flags");
  }();
  if (!flags) {  // sentinel hand-off (default); zbuf holds x
    if ((e = hipMemsetAsync(ybuf, 0xff, (size_t)N * sizeof(T), st)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(zbuf, 0xff, (size_t)N * sizeof(T), st)) != hipSuccess) return e;
    hipLaunchKernelGGL((trsv_sentinel_kernel<T, 64>), dim3(grid), dim3(PNT), 0, st, K, ld, N, D, Linv, b, ybuf, zbuf,
                       ctrl, nblk, skip);
    return hipGetLastError();
  }
  hipLaunchKernelGGL((trsv_persistent_kernel<T, 64>), dim3(grid), dim3(PNT), 0, st, K, ld, N, D, Linv, b, ybuf, zbuf,
                     ctrl, nblk, skip);
  return hipGetLastError();
}

hipError_t ldlt_solve_persistent(const double* K, int64_t ld, int N, const double* D, const double* Linv, int nbi,
                                 double* b, double* ybuf, double* zbuf, unsigned* ctrl, hipStream_t st) {
  return solve_persistent_t<double>(K, ld, N, D, Linv, nbi, b, ybuf, zbuf, ctrl, st);
}
hipError_t ldlt_solve_persistent(const float* K, int64_t ld, int N, const float* D, const float* Linv, int nbi,
                                 float* b, float* ybuf, float* zbuf, unsigned* ctrl, hipStream_t st,
                                 const unsigned* skip) {
  return solve_persistent_t<float>(K, ld, N, D, Linv, nbi, b, ybuf, zbuf, ctrl, st, skip);
}

}  // namespace ipmz
