// Reference point for the trailing-update GEMM: rocBLAS dgemm on the same
// shape (C R x R -= W L^T, rank nbo), full rectangle (2 R^2 nbo flops) --
// a measuring stick for gemm_nt_f64_kernel, not part of the product.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    auto _e = (x);                                                         \
    if ((int)_e) {                                                         \
      std::fprintf(stderr, "%s failed (%d) line %d\n", #x, (int)_e, __LINE__); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  rocblas_handle h;
  CK(rocblas_create_handle(&h));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  CK(rocblas_set_stream(h, st));
  for (int nbo : {256, 512}) {
    for (int R : {2048, 5632, 11008}) {
      const int64_t ld = (R + 63) / 64 * 64;
      double *C, *W, *L;
      CK(hipMalloc(&C, ld * R * 8));
      CK(hipMalloc(&W, (int64_t)R * nbo * 8));
      CK(hipMalloc(&L, ld * nbo * 8));
      CK(hipMemset(C, 0, ld * R * 8));
      CK(hipMemset(W, 0, (int64_t)R * nbo * 8));
      CK(hipMemset(L, 0, ld * nbo * 8));
      const double alpha = -1.0, beta = 1.0;
      // row-major C -= W L^T  ==  col-major C' -= L' W'^T ... as (T, N): C_cm(R x R) -= Lcm^T Wcm
      auto run = [&]() {
        CK(rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_none, R, R, nbo, &alpha, L, nbo, W, nbo,
                         &beta, C, ld));
      };
      run();
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      CK(hipEventRecord(a, st));
      const int reps = 5;
      for (int r = 0; r < reps; ++r) run();
      CK(hipEventRecord(b, st));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ms /= reps;
      std::printf("rocblas_dgemm R=%d k=%d: %.3f ms %.2f TFLOP/s (full 2R^2k)\n", R, nbo, ms,
                  2.0 * R * R * nbo / ms / 1e9);
      CK(hipFree(C));
      CK(hipFree(W));
      CK(hipFree(L));
    }
  }
  return 0;
}
