// Cross-workgroup hand-offs inside one launch (cdna_hip_programming.md §6
// Guideline 16, "Valid forms" row 1): data is stored write-through with
// relaxed agent-scope atomic stores (sc1) and read with agent-scope atomic
// loads, every storing wave drains vmcnt(0), a workgroup barrier, then ONE
// lane stores the flag with a relaxed agent-scope atomic.  The 8 XCDs have
// private L2s, so plain loads/stores are not enough for data that another
// workgroup of the same launch consumes.  A hand-off may also cross two
// concurrent launches of ONE kernel whose workgroups draw their roles from
// shared ticket counters (panel.hip), so a consumer never waits for a
// workgroup that has not been dispatched.
#pragma once
#include <hip/hip_runtime.h>

namespace ipmz {

// a wait gives up after this long (s_memrealtime runs at a constant 100 MHz):
// far beyond any legitimate hand-off, short enough that a bug surfaces as an
// error word instead of a hung queue
constexpr unsigned long long SPIN_TICKS = 50000000ull;  // 0.5 s

template <typename T>
__device__ __forceinline__ T ld_sc1(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one lane of the workgroup polls flag >= want; everyone leaves together.
// Gives up (and raises *err) after SPIN_TICKS or when *err is raised.
__device__ __forceinline__ bool wait_flag_ge(unsigned* flag, unsigned want, unsigned* err, unsigned* sh_ok) {
  if (threadIdx.x == 0) {
    unsigned ok = 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS ||
          __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    *sh_ok = ok;
  }
  __syncthreads();
  return *sh_ok != 0;
}
__device__ __forceinline__ bool wait_flag(unsigned* flag, unsigned* err, unsigned* sh_ok) {
  return wait_flag_ge(flag, 1u, err, sh_ok);
}

// lanes 0 .. n-1 of wave 0 poll flags base[0 .. n-1] >= 1 together (one L2
// round trip per try for all of them) and lane 63 samples *peek (no wait:
// *sh_peek = whether it was up); everyone leaves together.  Gives up as
// wait_flag_ge does.
__device__ __forceinline__ bool wait_flags(unsigned* base, int n, const unsigned* peek, unsigned* err, unsigned* sh_ok,
                                           unsigned* sh_peek) {
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    unsigned ok = 1, pk = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      const unsigned v = l < n ? __hip_atomic_load(&base[l], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 1u;
      if (l == 63 && peek && !pk) pk = __hip_atomic_load(peek, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__builtin_amdgcn_ballot_w64(v == 0u) == 0ull) break;
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_TICKS ||
          __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
        if (l == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    if (l == 0) *sh_ok = ok;
    if (l == 63) *sh_peek = pk != 0u;
  }
  __syncthreads();
  return *sh_ok != 0;
}

// every storing wave drains its sc1 stores, then one lane raises the flag
__device__ __forceinline__ void publish(unsigned* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace ipmz
