// Shared definitions for the gfx950 (MI355X, CDNA4) kernels of libipmz.
//
// Storage conventions (DESIGN.md "Data layout in HBM"):
//   * dense matrices are row-major with a leading dimension `ld` (elements);
//   * the KKT matrix K is symmetric and only its LOWER triangle (i >= j) is
//     read; the LDL^T factor overwrites the strict lower triangle with L
//     (unit diagonal implicit) and writes D to a separate vector.  Row-major
//     lower == column-major upper, so the reference's row-major Matrix
//     (LinearSolvers.cpp:14-42) maps onto it by a plain copy.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#define IPMZ_HOST_DEVICE __host__ __device__ __forceinline__

typedef double double4_t __attribute__((ext_vector_type(4)));

// hipcc builds this library with -ffp-contract=off: element-wise Newton
// formulas then round exactly like the reference evaluator
// (Evaluation.cpp:202-257); the dense kernels use explicit fma / MFMA.

// Evaluation.cpp:267-271 -- element-wise reciprocal, 0 -> sqrt(DBL_MAX).
IPMZ_HOST_DEVICE double ipmz_inv(double x) {
  return x == 0.0 ? 1.3407807929942596e+154 : 1.0 / x;
}

// Counter-based splitmix64 generator, identical to
// oracle/ipmz_oracle.cpp so GPU-generated inputs match the oracle bitwise.
IPMZ_HOST_DEVICE uint64_t ipmz_splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
IPMZ_HOST_DEVICE double ipmz_u01(uint64_t seed, uint64_t tag, uint64_t i, uint64_t j) {
  const uint64_t key = seed ^ (tag << 56) ^ ((i << 32) + j);
  return (double)(ipmz_splitmix64(key) >> 11) * 0x1.0p-53;
}

__device__ __forceinline__ double4_t mfma_f64_16x16x4(double a, double b, double4_t c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// One MFMA shape for both precisions of the factorization: 16 x 16 x 4 with
// A/B fragments (row l & 15, k l >> 4) -- identical for f64 and f32 -- and
// the accumulator map that differs: f64 rows (l >> 4) + 4 r, f32 rows
// 4 (l >> 4) + r (cdna_hip_programming.md §3; the f32 form is an exact f32
// fma chain at 2x the f64 rate, 32 vs 64 cycles per instruction).
typedef float float4_t __attribute__((ext_vector_type(4)));
template <typename T>
struct Mfma;
template <>
struct Mfma<double> {
  typedef double4_t acc_t;
  typedef double2 vec2_t;
  static __device__ __forceinline__ acc_t mma(double a, double b, acc_t c) { return mfma_f64_16x16x4(a, b, c); }
  static __device__ __forceinline__ int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};
template <>
struct Mfma<float> {
  typedef float4_t acc_t;
  typedef float2 vec2_t;
  static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ int row(int lane, int r) { return 4 * (lane >> 4) + r; }
};

// Wave-level all-reductions (wave64) on the VALU: DPP inside 16-lane rows
// (xor 1, xor 2, rotate 4, rotate 8), then v_permlane16_swap / 32_swap across
// rows (gfx950).  No LDS round trips (ds_bpermute-based __shfl_xor costs ~6
// dependent LDS latencies for a double).
template <int CTRL>
__device__ __forceinline__ double dpp_double(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
// lane-broadcast DPP (row_newbcast etc.): no old value, so no v_mov of a
// placeholder before every v_mov_dpp
template <int CTRL>
__device__ __forceinline__ double dpp_bcast(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
// 1/d from v_rcp_f64 and two Newton steps (5 dependent ops instead of the
// 10-op IEEE division sequence); finite nonzero d only
__device__ __forceinline__ double fast_rcp(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
}
template <int CTRL>
__device__ __forceinline__ float dpp_float(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_t(double v) { return dpp_double<CTRL>(v); }
template <int CTRL>
__device__ __forceinline__ float dpp_t(float v) { return dpp_float<CTRL>(v); }
__device__ __forceinline__ double readlane_t(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ float readlane_t(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ void swap16(double v, double& a, double& b) {
  const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
  a = __hiloint2double(hi[0], lo[0]);
  b = __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ void swap32(double v, double& a, double& b) {
  const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
  a = __hiloint2double(hi[0], lo[0]);
  b = __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_double<0xb1>(v);   // quad_perm [1,0,3,2]
  v += dpp_double<0x4e>(v);   // quad_perm [2,3,0,1]
  v += dpp_double<0x124>(v);  // row_ror:4
  v += dpp_double<0x128>(v);  // row_ror:8
  double a, b;
  swap16(v, a, b);
  v = a + b;
  swap32(v, a, b);
  return a + b;
}
__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, dpp_double<0xb1>(v));
  v = fmax(v, dpp_double<0x4e>(v));
  v = fmax(v, dpp_double<0x124>(v));
  v = fmax(v, dpp_double<0x128>(v));
  double a, b;
  swap16(v, a, b);
  v = fmax(a, b);
  swap32(v, a, b);
  return fmax(a, b);
}
__device__ __forceinline__ double wave_min(double v) {
  v = fmin(v, dpp_double<0xb1>(v));
  v = fmin(v, dpp_double<0x4e>(v));
  v = fmin(v, dpp_double<0x124>(v));
  v = fmin(v, dpp_double<0x128>(v));
  double a, b;
  swap16(v, a, b);
  v = fmin(a, b);
  swap32(v, a, b);
  return fmin(a, b);
}

// compile-time loop: f(std::integral_constant<int, I>{}) for I in [0, N),
// for bodies that must index register arrays with constants
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// compute units of the current device (cached per process; one device type)
inline int device_cus() {
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  return cus;
}

