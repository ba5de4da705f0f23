// fp32 trailing-update micro-benchmark (the C5 factor's C -= W L^T, rank
// 512): the product's sgemm_nt_kernel tile variants (csrc/gemm32.h) against
// the previous engine instance (gemm.h) and rocBLAS SGEMM / SSYRKX, on the
// product's operand layout (L and C inside one row-major matrix, ld = 16384),
// each checked against an fp64 recomputation of sampled rows.
// Tool only (links rocBLAS as a measuring stick; the product does not).
//   build: make -C ipm-zoo_amd sgemmbench ; run: ipm-zoo_amd/build/sgemm_bench [R] [variants...]
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"
#include "gemm.h"
#include "gemm32.h"
#include "gemm64.h"

#define CK(x)                                                                             \
  do {                                                                                    \
    auto _e = (x);                                                                        \
    if ((int)_e) {                                                                        \
      std::fprintf(stderr, "%s:%d %s failed (%d)\n", __FILE__, __LINE__, #x, (int)_e);    \
      std::exit(1);                                                                       \
    }                                                                                     \
  } while (0)

using namespace ipmz;

template <typename T>
__global__ void fill_u(T* P, int64_t n, uint64_t seed) {
  for (int64_t t = blockIdx.x * 256ll + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256)
    P[t] = (T)(2.0 * ipmz_u01(seed, 3, (uint64_t)(t >> 24), (uint64_t)(t & 0xffffff)) - 1.0);
}
// err[i'] = max_j |C[i][j] - (C0[i][j] - sum_k W[i][k] L[j][k])| / sum_k |W L| over the rows i = i' * rs, j <= i
template <typename T>
__global__ void check_rows(const T* C, const T* C0, int64_t ldc, const T* W, int64_t ldw, const T* L,
                           int64_t ldl, int R, int N, int k, int rs, int lowtri, double* err) {
  const int i = blockIdx.x * rs;
  if (i >= R) return;
  double e = 0.0;
  // lowtri 1: the triangle (j <= i); 0: a strip (tiles above the diagonal skipped, so j <= i); 2: every column
  const int jend = lowtri == 2 ? N : (i + 1 < N ? i + 1 : N);
  for (int j = threadIdx.x; j < jend; j += blockDim.x) {
    double s = 0.0, a = 0.0;
    for (int q = 0; q < k; ++q) {
      const double p = (double)W[(int64_t)i * ldw + q] * (double)L[(int64_t)j * ldl + q];
      s += p;
      a += fabs(p);
    }
    const double ref = (double)C0[(int64_t)i * ldc + j] - s;
    const double d = fabs((double)C[(int64_t)i * ldc + j] - ref) / (a + 1e-30);
    e = d > e ? d : e;
  }
  __shared__ double red[256];
  red[threadIdx.x] = e;
  __syncthreads();
  for (int s = 128; s; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) err[blockIdx.x] = red[0];
}

static hipError_t run_variant(int v, GemmArgsT<double> g, hipStream_t st) {
  hipError_t e = hipSuccess;
  switch (v) {
    case 0: return launch_gemm<128, 128, EPI_SUB, 4, 4, OPT_NOR2 | OPT_GRP>(g, st);  // the product's fp64 trailing tile
    case 1: return launch_dgemm_glds<128, 128, 4, 4, 8, 3, 8>(g, st, e) ? e : hipErrorInvalidValue;
    case 2: return launch_dgemm_glds<128, 128, 4, 4, 16, 2, 8>(g, st, e) ? e : hipErrorInvalidValue;
    case 3: return launch_dgemm_glds<128, 128, 2, 4, 8, 3, 4>(g, st, e) ? e : hipErrorInvalidValue;
    case 4: return launch_dgemm_glds<128, 128, 2, 4, 16, 2, 4>(g, st, e) ? e : hipErrorInvalidValue;
    case 5: return launch_dgemm_glds<128, 128, 4, 4, 16, 3, 4>(g, st, e) ? e : hipErrorInvalidValue;
    case 6: return launch_dgemm_glds<128, 128, 2, 4, 16, 3, 4>(g, st, e) ? e : hipErrorInvalidValue;
    case 7: return launch_dgemm_glds<256, 128, 4, 4, 16, 2, 4>(g, st, e) ? e : hipErrorInvalidValue;
    case 8: return launch_dgemm_glds<64, 64, 2, 2, 8, 3, 8, EPI_SUB_STRIP>(g, st, e) ? e : hipErrorInvalidValue;
    case 9: return launch_dgemm_glds<64, 128, 2, 2, 8, 3, 4, EPI_SUB_STRIP>(g, st, e) ? e : hipErrorInvalidValue;
    case 10: return launch_gemm<64, 64, EPI_SUB_STRIP, 2, 2, OPT_NOR2>(g, st);   // the product's strip tiles
    case 11: return launch_gemm<64, 128, EPI_SUB_STRIP, 2, 4, OPT_NOR2>(g, st);
    case 12: return launch_gemm<128, 128, EPI_SUB_STRIP, 2, 4, OPT_NOR2>(g, st);
    default: return hipErrorInvalidValue;
  }
}
static hipError_t run_variant(int v, GemmArgsT<float> g, hipStream_t st) {
  switch (v) {
    case 0: return launch_gemm<128, 128, EPI_SUB, 2, 4, OPT_NOR2 | OPT_GRP>(g, st);  // round-3 hand-written fp32
    case 1: return launch_sgemm<128, 128, 2, 2, 32, 2>(g, st);
    case 2: return launch_sgemm<128, 128, 2, 2, 16, 2>(g, st);
    case 3: return launch_sgemm<256, 128, 4, 2, 16, 2>(g, st);
    case 4: return launch_sgemm<256, 256, 4, 4, 16, 4>(g, st);
    case 5: return launch_sgemm<128, 128, 2, 4, 32, 4>(g, st);
    case 6: return launch_sgemm<128, 128, 2, 4, 16, 4>(g, st);
    case 7: return launch_sgemm<256, 256, 4, 4, 32, 4>(g, st);
    case 8: return launch_sgemm<128, 256, 2, 4, 16, 4>(g, st);
    case 9: return launch_sgemm<64, 64, 2, 2, 32, 4>(g, st);
    case 10: return launch_sgemm<128, 128, 2, 2, 16, 4>(g, st);
    // LDS-DMA staging (global_load_lds), NST-deep ring
    case 11: return launch_sgemm<128, 128, 2, 4, 16, 4, EPI_SUB, 3>(g, st);
    case 12: return launch_sgemm<128, 128, 2, 2, 16, 2, EPI_SUB, 3>(g, st);
    case 13: return launch_sgemm<128, 128, 2, 4, 32, 4, EPI_SUB, 3>(g, st);
    case 14: return launch_sgemm<128, 128, 2, 2, 32, 2, EPI_SUB, 3>(g, st);
    case 15: return launch_sgemm<256, 128, 4, 2, 16, 2, EPI_SUB, 3>(g, st);
    case 16: return launch_sgemm<256, 256, 4, 4, 16, 2, EPI_SUB, 3>(g, st);
    case 17: return launch_sgemm<128, 128, 2, 4, 16, 4, EPI_SUB, 2>(g, st);
    case 18: return launch_sgemm<128, 128, 2, 4, 32, 4, EPI_SUB, 2>(g, st);
    // LDS-DMA + fragment reads in asm
    case 21: return launch_sgemm<128, 128, 2, 4, 16, 4, EPI_SUB, 3, true>(g, st);
    case 22: return launch_sgemm<128, 128, 2, 2, 16, 2, EPI_SUB, 3, true>(g, st);
    case 23: return launch_sgemm<128, 128, 2, 4, 32, 4, EPI_SUB, 3, true>(g, st);
    case 25: return launch_sgemm<256, 128, 4, 2, 16, 2, EPI_SUB, 3, true>(g, st);
    case 26: return launch_sgemm<256, 256, 4, 4, 16, 2, EPI_SUB, 3, true>(g, st);
    case 27: return launch_sgemm<128, 128, 2, 2, 16, 2, EPI_SUB, 2, true>(g, st);
    case 28: return launch_sgemm<128, 128, 2, 2, 32, 2, EPI_SUB, 2, true>(g, st);
    default: return hipErrorInvalidValue;
  }
}

template <typename T>
static int run_all(int R, std::vector<int> vars) {
  const int k = 512;
  constexpr bool F32 = sizeof(T) == 4;
  if (vars.empty()) {
    if (F32) vars = {0, 10, 21, 22, 27, 28, 100, 101};
    else vars = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 100};
  }
  const int Nt = R + k;
  const int64_t ld = (Nt + 63) / 64 * 64;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  T *K, *K0, *W;
  CK(hipMalloc(&K, ld * Nt * sizeof(T)));
  CK(hipMalloc(&K0, ld * Nt * sizeof(T)));
  CK(hipMalloc(&W, (int64_t)R * k * sizeof(T)));
  hipLaunchKernelGGL(fill_u<T>, dim3(4096), dim3(256), 0, st, K0, ld * Nt, 11ull);
  hipLaunchKernelGGL(fill_u<T>, dim3(4096), dim3(256), 0, st, W, (int64_t)R * k, 12ull);
  const T* L = K + (int64_t)k * ld;  // rows k.., columns 0..k-1
  T* C = K + (int64_t)k * ld + k;
  const int rs = 61, nrows = (R + rs - 1) / rs;
  double* err;
  CK(hipMalloc(&err, nrows * 8));
  std::vector<double> herr(nrows);
  rocblas_handle h;
  CK(rocblas_create_handle(&h));
  CK(rocblas_set_stream(h, st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int shape = 0; shape < 3; ++shape) {
    // shape 0: the trailing triangle R x R; shape 1: a look-ahead strip, R rows x 512 columns;
    // shape 2: the full square R x R (every tile; rocBLAS SGEMM's shape), flops 2 R^2 k
    const int Ncols = shape == 1 ? 512 : R;
    const double fl = shape == 0 ? (double)R * (R + 1) * k : 2.0 * R * Ncols * k;
    for (int v : vars) {
      if (shape == 1 && v >= 100) continue;
      if (shape == 2 && v == 100) continue;
      if (!F32 && v >= 100 && shape != 0) continue;
      GemmArgsT<T> g{};
      g.M = R;
      g.N = Ncols;
      g.Kd = k;
      g.A = W;
      g.lda = k;
      g.B = L;
      g.ldb = ld;
      g.C = C;
      g.ldc = ld;
      g.lower = shape == 0 ? 2 : shape == 1 ? 1 : 0;
      g.row0 = shape == 0 ? 0 : 0;
      g.col0 = 0;
      const T alpha = -1, beta = 1;
      auto run = [&]() -> int {
        if constexpr (F32) {
          if (v == 100)
            return (int)rocblas_ssyrkx(h, rocblas_fill_upper, rocblas_operation_transpose, R, k, &alpha, L, (int)ld, W,
                                       k, &beta, C, (int)ld);
          if (v == 101)  // the full square (2 R^2 k, reported per R(R+1)k like the others)
            return (int)rocblas_sgemm(h, rocblas_operation_transpose, rocblas_operation_none, R, R, k, &alpha, L,
                                      (int)ld, W, k, &beta, C, (int)ld);
        } else {
          if (v == 100)  // rocBLAS DGEMM on the full square (2 R^2 k, reported per R(R+1)k like the others)
            return (int)rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_none, R, R, k, &alpha, L,
                                      (int)ld, W, k, &beta, C, (int)ld);
        }
        return (int)run_variant(v, g, st);
      };
      CK(hipMemcpyAsync(K, K0, ld * Nt * sizeof(T), hipMemcpyDeviceToDevice, st));
      if (run()) {
        std::printf("variant %d: launch failed\n", v);
        continue;
      }
      // check (rocBLAS rows: the column-major upper = row-major lower too)
      hipLaunchKernelGGL(check_rows<T>, dim3(nrows), dim3(256), 0, st, C, K0 + (int64_t)k * ld + k, ld, W, (int64_t)k, L,
                         ld, R, Ncols, k, rs, shape == 2 ? 2 : shape == 0 ? 1 : 0, err);
      CK(hipMemcpyAsync(herr.data(), err, nrows * 8, hipMemcpyDeviceToHost, st));
      CK(hipStreamSynchronize(st));
      double me = 0.0;
      for (double x : herr) me = x > me ? x : me;
      const int reps = 5;
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) run();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      std::printf("%s %s R=%5d k=%d variant %3d: %.3f ms %7.2f TFLOP/s  max rel err %.2e\n", F32 ? "f32" : "f64",
                  shape == 0 ? "trailing" : shape == 1 ? "strip   " : "square  ", R, k, v, ms, fl / ms / 1e9, me);
    }
  }
  return 0;
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  // sgemm_bench [R] [variants...]: fp32; sgemm_bench d [R] [variants...]: fp64
  int a = 1;
  const bool f64 = argc > 1 && argv[1][0] == 'd';
  if (f64) ++a;
  const int R = argc > a ? std::atoi(argv[a]) : (f64 ? 10752 : 15872);
  std::vector<int> vars;
  for (int i = a + 1; i < argc; ++i) vars.push_back(std::atoi(argv[i]));
  return f64 ? run_all<double>(R, vars) : run_all<float>(R, vars);
}
