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

// fp32 (the mixed-precision factor's trailing update): rocblas_sgemm on the
// full square and rocblas_ssyrkx on the lower triangle (R^2 k flops counted)
static void fp32(rocblas_handle h, hipStream_t st) {
  for (int R : {8192, 15872}) {
    const int nbo = 512;
    const int64_t ld = (R + 63) / 64 * 64;
    float *C, *W, *L;
    CK(hipMalloc(&C, ld * R * 4));
    CK(hipMalloc(&W, (int64_t)R * nbo * 4));
    CK(hipMalloc(&L, (int64_t)R * nbo * 4));
    CK(hipMemset(C, 0, ld * R * 4));
    CK(hipMemset(W, 0, (int64_t)R * nbo * 4));
    CK(hipMemset(L, 0, (int64_t)R * nbo * 4));
    const float alpha = -1.f, beta = 1.f;
    for (int which = 0; which < 2; ++which) {
      auto run = [&]() {
        if (which == 0)
          CK(rocblas_sgemm(h, rocblas_operation_transpose, rocblas_operation_none, R, R, nbo, &alpha, L, nbo, W, nbo,
                           &beta, C, ld));
        else  // col-major upper of C' = lower of row-major C: C' -= L'^T W' (op T)
          CK(rocblas_ssyrkx(h, rocblas_fill_upper, rocblas_operation_transpose, R, nbo, &alpha, L, nbo, W, nbo, &beta,
                            C, ld));
      };
      run();
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      CK(hipEventRecord(a, st));
      for (int r = 0; r < 5; ++r) run();
      CK(hipEventRecord(b, st));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ms /= 5;
      const double fl = which == 0 ? 2.0 * R * R * nbo : (double)R * (R + 1) * nbo;
      std::printf("%s R=%d k=%d: %.3f ms %.2f TFLOP/s (%s)\n", which == 0 ? "rocblas_sgemm " : "rocblas_ssyrkx", R, nbo,
                  ms, fl / ms / 1e9, which == 0 ? "full 2R^2k" : "lower R(R+1)k");
    }
    CK(hipFree(C));
    CK(hipFree(W));
    CK(hipFree(L));
  }
}

// fp64 SYRKX on the C3 trailing shapes (R(R+1)k flops counted)
static void fp64syrkx(rocblas_handle h, hipStream_t st) {
  for (int R : {5632, 10752}) {
    const int nbo = 512;
    const int64_t ld = (R + 63) / 64 * 64;
    double *C, *W, *L;
    CK(hipMalloc(&C, ld * R * 8));
    CK(hipMalloc(&W, (int64_t)R * nbo * 8));
    CK(hipMalloc(&L, (int64_t)R * nbo * 8));
    CK(hipMemset(C, 0, ld * R * 8));
    CK(hipMemset(W, 0, (int64_t)R * nbo * 8));
    CK(hipMemset(L, 0, (int64_t)R * nbo * 8));
    const double alpha = -1.0, beta = 1.0;
    auto run = [&]() {
      CK(rocblas_dsyrkx(h, rocblas_fill_upper, rocblas_operation_transpose, R, nbo, &alpha, L, nbo, W, nbo, &beta, C,
                        ld));
    };
    run();
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, st));
    for (int r = 0; r < 5; ++r) run();
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= 5;
    std::printf("rocblas_dsyrkx R=%d k=%d: %.3f ms %.2f TFLOP/s (lower R(R+1)k)\n", R, nbo, ms,
                (double)R * (R + 1) * nbo / ms / 1e9);
    CK(hipFree(C));
    CK(hipFree(W));
    CK(hipFree(L));
  }
}

int main(int argc, char** argv) {
  rocblas_handle h;
  CK(rocblas_create_handle(&h));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  CK(rocblas_set_stream(h, st));
  if (argc > 1 && argv[1][0] == 's') {
    fp32(h, st);
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'x') {
    fp64syrkx(h, st);
    return 0;
  }
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
