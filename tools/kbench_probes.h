// Experiment kernels of tools/kbench (not part of libipmz).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ipmz {
hipError_t gemm_nt_sub_variant(int variant, int M, int N, int Kd, const double* A, int64_t lda, const double* B,
                               int64_t ldb, double* C, int64_t ldc, hipStream_t st);
hipError_t gemm_nt_sub_variant32(int variant, int M, int N, int Kd, const float* A, int64_t lda, const float* B,
                                 int64_t ldb, float* C, int64_t ldc, hipStream_t st);
hipError_t mfma_probe(double* out, int blocks, int iters, int threads, int nacc, hipStream_t st);
hipError_t diag_clock_probe(double* K, int64_t ld, double* D, double* Linv, int* info, unsigned long long* out,
                            hipStream_t st, int cpv = 0);
}  // namespace ipmz
