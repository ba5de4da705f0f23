// Experiment kernels for tools/kbench.cpp (NOT part of libipmz): tile
// variants of the product GEMM engine (csrc/gemm.h), an f64 MFMA throughput
// probe and stage clocks of the 64 x 64 diagonal factor (csrc/diag64.h).
#include "common.h"
#include "diag64.h"
#include "gemm.h"
#include "kbench_probes.h"

namespace ipmz {

hipError_t gemm_nt_sub_variant(int variant, int M, int N, int Kd, const double* A, int64_t lda, const double* B,
                               int64_t ldb, double* C, int64_t ldc, hipStream_t st) {
  GemmArgs g{};
  g.M = M;
  g.N = N;
  g.Kd = Kd;
  g.A = A;
  g.lda = lda;
  g.B = B;
  g.ldb = ldb;
  g.C = C;
  g.ldc = ldc;
  g.lower = 2;
  switch (variant) {
    case 0: return launch_gemm<128, 128, EPI_SUB>(g, st);
    case 1: return launch_gemm<256, 128, EPI_SUB, 4, 2>(g, st);
    case 2: return launch_gemm<128, 128, EPI_SUB, 2, 4, 0>(g, st);
    case 4: return launch_gemm<256, 128, EPI_SUB, 4, 4>(g, st);
    case 5: return launch_gemm<128, 128, EPI_SUB, 4, 4>(g, st);
    case 6: return launch_gemm<128, 256, EPI_SUB, 2, 8>(g, st);
    case 14: return launch_gemm<128, 128, EPI_SUB, 2, 4, OPT_NOR2 | OPT_GRP>(g, st);
    case 15: return launch_gemm<128, 128, EPI_SUB, 4, 4, OPT_NOR2 | OPT_GRP>(g, st);  // the product's trailing tile
    case 23: return launch_gemm<64, 64, EPI_SUB, 2, 2, OPT_NOR2 | OPT_GRP>(g, st);
    // persistent grids (OPT_PERSIST): 16-wave tile with 256 / 384 / 512 workgroups
    case 30: g.persist = 256; return launch_gemm<128, 128, EPI_SUB, 4, 4, OPT_NOR2 | OPT_GRP | OPT_PERSIST>(g, st);
    case 31: g.persist = 384; return launch_gemm<128, 128, EPI_SUB, 4, 4, OPT_NOR2 | OPT_GRP | OPT_PERSIST>(g, st);
    case 32: g.persist = 512; return launch_gemm<128, 128, EPI_SUB, 4, 4, OPT_NOR2 | OPT_GRP | OPT_PERSIST>(g, st);
    case 33: g.persist = 248; return launch_gemm<128, 128, EPI_SUB, 4, 4, OPT_NOR2 | OPT_GRP | OPT_PERSIST>(g, st);
    default: break;
  }
  g.lower = 1;  // strip (rectangle, upper tiles of the diagonal band skipped)
  switch (variant) {
    case 20: return launch_gemm<128, 128, EPI_SUB_STRIP, 2, 4, OPT_NOR2>(g, st);
    case 21: return launch_gemm<64, 64, EPI_SUB_STRIP, 2, 2, OPT_NOR2>(g, st);
    case 22: return launch_gemm<64, 128, EPI_SUB_STRIP, 2, 4, OPT_NOR2>(g, st);
    case 24: return launch_gemm<128, 128, EPI_SUB_STRIP, 4, 4, OPT_NOR2>(g, st);
    default: break;
  }
  g.lower = 2;
  switch (variant) {  // stage depth BK = 32 (half the barriers per k)
    case 40: return launch_gemm<128, 128, EPI_SUB, 4, 4, OPT_NOR2 | OPT_GRP, 32>(g, st);
    case 41: return launch_gemm<128, 128, EPI_SUB, 2, 4, OPT_NOR2 | OPT_GRP, 32>(g, st);
    default: return hipErrorInvalidValue;
  }
}

// fp32 trailing-update variants (the mixed-precision factor, C5)
hipError_t gemm_nt_sub_variant32(int variant, int M, int N, int Kd, const float* A, int64_t lda, const float* B,
                                 int64_t ldb, float* C, int64_t ldc, hipStream_t st) {
  GemmArgsT<float> g{};
  g.M = M;
  g.N = N;
  g.Kd = Kd;
  g.A = A;
  g.lda = lda;
  g.B = B;
  g.ldb = ldb;
  g.C = C;
  g.ldc = ldc;
  g.lower = 2;
  switch (variant) {
    case 0: return launch_gemm<128, 128, EPI_SUB, 2, 4, OPT_NOR2 | OPT_GRP>(g, st);  // the product's fp32 tile
    case 1: return launch_gemm<128, 128, EPI_SUB, 4, 4, OPT_NOR2 | OPT_GRP>(g, st);
    case 2: return launch_gemm<128, 128, EPI_SUB, 2, 4, OPT_NOR2 | OPT_GRP, 32>(g, st);
    case 3: return launch_gemm<128, 128, EPI_SUB, 4, 4, OPT_NOR2 | OPT_GRP, 32>(g, st);
    case 4: return launch_gemm<128, 128, EPI_SUB, 2, 4, OPT_GRP, 32>(g, st);
    case 5: return launch_gemm<128, 128, EPI_SUB, 2, 4, OPT_NOR2 | OPT_GRP, 64>(g, st);
    case 6: return launch_gemm<256, 256, EPI_SUB, 4, 4, OPT_NOR2 | OPT_GRP, 16>(g, st);
    case 7: return launch_gemm<256, 256, EPI_SUB, 4, 4, OPT_NOR2 | OPT_GRP, 32>(g, st);
    default: return hipErrorInvalidValue;
  }
}

// f64 MFMA throughput: each wave runs `iters` x NACC independent
// v_mfma_f64_16x16x4 on register data
template <int NACC>
__global__ __launch_bounds__(512) void mfma_probe_kernel(double* out, int iters) {
  double4_t acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = (double4_t){0.0, 0.0, 0.0, 0.0};
  double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = mfma_f64_16x16x4(a, b, acc[i]);
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[0] = s;
}
hipError_t mfma_probe(double* out, int blocks, int iters, int threads, int nacc, hipStream_t st) {
  if (nacc == 16) hipLaunchKernelGGL(mfma_probe_kernel<16>, dim3(blocks), dim3(threads), 0, st, out, iters);
  else if (nacc == 8) hipLaunchKernelGGL(mfma_probe_kernel<8>, dim3(blocks), dim3(threads), 0, st, out, iters);
  else if (nacc == 1) hipLaunchKernelGGL(mfma_probe_kernel<1>, dim3(blocks), dim3(threads), 0, st, out, iters);
  else hipLaunchKernelGGL(mfma_probe_kernel<4>, dim3(blocks), dim3(threads), 0, st, out, iters);
  return hipGetLastError();
}

// stage clocks (s_memtime) of one diag64_body run: entries [0, clk[31]) of out
__device__ unsigned long long g_diag_clk[32];
template <int CPV, bool COH>
__global__ __launch_bounds__(256) void diag_clock_kernel(double* K, int64_t ld, double* D, double* Linv, int* info) {
  __shared__ double M[64 * DS], X[64 * DS], dsh[64];
  diag64_body<COH, false, double, false, 4, NoHook, true, NoHook, CPV>(K, ld, 0, 64, D, Linv, info, M, X, dsh,
                                                                      g_diag_clk);
}
// v: CPV (0 colpass16, 1 colpass16_spec, 3 / 4 colpass16_short with 2 / 1 Newton steps) + 8 COH (L^{-1}
// stored write-through, as the panel chain)
hipError_t diag_clock_probe(double* K, int64_t ld, double* D, double* Linv, int* info, unsigned long long* out,
                            hipStream_t st, int v) {
#define DCK(C, H) \
  if (v == (C) + ((H) ? 8 : 0)) hipLaunchKernelGGL((diag_clock_kernel<C, H>), dim3(1), dim3(256), 0, st, K, ld, D, Linv, info)
  DCK(0, false);
  DCK(1, false);
  DCK(1, true);
  DCK(3, true);
  DCK(4, true);
#undef DCK
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return hipMemcpyFromSymbolAsync(out, HIP_SYMBOL(g_diag_clk), sizeof(unsigned long long) * 32, 0,
                                  hipMemcpyDeviceToHost, st);
}

}  // namespace ipmz
