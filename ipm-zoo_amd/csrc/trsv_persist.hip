// Single-launch, sync-free triangular solve with the LDL^T factor:
//   x = L^{-T} D^{-1} L^{-1} b   (LinearSolvers.cpp:44-74)
//
// The forward sweep (Ly = b) and the backward sweep (L^T x = D^{-1} y) are
// 2 * nblk "tickets" of NB-row blocks, claimed in dependency order from a
// device counter by whichever workgroup is running (dequeue pattern): a
// ticket only ever waits on LOWER tickets, all of which belong to running
// workgroups, so the grid cannot deadlock whatever the dispatch order.
//
//   forward block J  : v = b_J - sum_{K<J} L_JK y_K ; y_J = Linv_J v
//   backward block J : u = y_J / D_J - sum_{K>J} L_KJ^T x_K ; x_J = Linv_J^T u
// Every off-diagonal tile is streamed into registers BEFORE the vector it
// needs is polled, so the critical path per block is one hand-off plus one
// NB x NB tile product plus the diagonal-block apply.
//
// Hand-off: the block vectors y and x start as an all-ones bit pattern (a NaN
// payload arithmetic never produces) and are stored write-through (sc1); a
// consumer polls the 64 elements with agent-scope loads until none is the
// sentinel -- one aligned 8-byte store per element, so seeing it is seeing
// its final value (MI355X_MICROARCH.md, R2 granule).  Spins are bounded: on
// timeout the kernel raises ctrl[1], a STICKY error word (cleared only when
// a factorization starts) that the host folds into its return codes.
#include "common.h"
#include "kernels.h"
#include "sync.h"


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

// ---------------------------------------------------------------------------
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
                                                            const unsigned* __restrict__ skip, int inject) {
  typedef typename Mfma<T>::vec2_t V2;
  if (skip && *skip) return;  // mixed-precision refinement already converged
  static_assert(NB == 64, "persistent solve is written for 64-row blocks");
  __shared__ T vec[NB];
  __shared__ T red[4][NB];
  __shared__ unsigned sh_ticket, sh_ok;
  unsigned* counter = ctrl;
  unsigned* err = ctrl + SOLVE_ERR_WORD;
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
      // inject (tests only): block 0 never publishes -> every consumer times out
      if ((tid & 3) == 0 && r < rows && !(inject && J == 0)) st_sc1(&ybuf[J0 + r], y);
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
                                     T* xbuf, unsigned* ctrl, hipStream_t st, const unsigned* skip = nullptr) {
  if (N <= 0) return hipSuccess;
  if (nbi != 64) return hipErrorInvalidValue;
  const int nblk = (N + 63) / 64;
  // the ticket counter only: ctrl[1] (error) stays sticky
  hipError_t e = hipMemsetAsync(ctrl, 0, sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  if ((e = hipMemsetAsync(ybuf, 0xff, (size_t)N * sizeof(T), st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(xbuf, 0xff, (size_t)N * sizeof(T), st)) != hipSuccess) return e;
  // resident grid: 3 workgroups per CU fit (LDS ~2.6 KB, < 128 VGPRs); the
  // dequeue makes residency a performance matter only
  const int grid = 2 * nblk < 512 ? 2 * nblk : 512;
  hipLaunchKernelGGL((trsv_sentinel_kernel<T, 64>), dim3(grid), dim3(PNT), 0, st, K, ld, N, D, Linv, b, ybuf, xbuf,
                     ctrl, nblk, skip, debug_inject_mask() & IPMZ_INJECT_SOLVE);
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
