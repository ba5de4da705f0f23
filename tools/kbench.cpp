// Kernel micro-benchmark for libipmz (MI355X): times the factor pieces with
// HIP events.  Build: make -C ipm-zoo_amd kbench ; run: ipm-zoo_amd/build/kbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "common.h"
#include "kernels.h"

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e = (x);                                                                    \
    if (e != hipSuccess) {                                                                 \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

__global__ void fill_qd(double* K, int64_t ld, int N, unsigned long long seed) {
  const int64_t total = (int64_t)N * N;
  for (int64_t t = blockIdx.x * 256ll + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t i = t / N, j = t % N;
    const int64_t a = i > j ? i : j, b = i > j ? j : i;
    double v = (2.0 * ipmz_u01(seed, 9, a, b) - 1.0) / (double)N;
    if (i == j) v = (i < 3 * N / 4) ? 1.0 + ipmz_u01(seed, 9, i, i) : -(0.5 + ipmz_u01(seed, 9, i, i));
    K[i * ld + j] = v;
  }
}

struct Timer {
  hipEvent_t a, b;
  Timer() {
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
  }
  void start(hipStream_t s) { CK(hipEventRecord(a, s)); }
  float stop(hipStream_t s) {
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms;
  }
};

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int N = argc > 1 ? std::atoi(argv[1]) : 11264;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const int64_t ld = (N + 63) / 64 * 64;
  double *K, *D, *Linv, *W, *b, *side;
  int* info;
  CK(hipMalloc(&K, ld * N * 8));
  CK(hipMalloc(&D, N * 8));
  CK(hipMalloc(&Linv, (int64_t)(N + 127) / 64 * 128 * 128 * 8));
  CK(hipMalloc(&W, 3ll * N * 512 * 8));
  CK(hipMalloc(&b, N * 8));
  CK(hipMalloc(&side, 1024 * 8));
  CK(hipMalloc(&info, 64));
  double *yb, *zb;
  unsigned* ctrl;
  CK(hipMalloc(&yb, N * 8));
  CK(hipMalloc(&zb, N * 8));
  CK(hipMalloc(&ctrl, (2 + 2 * (N + 63) / 64) * 4 + 256));
  unsigned* pctrl;
  CK(hipMalloc(&pctrl, IPMZ_PANEL_CTRL_WORDS * 4));
  CK(hipMemset(pctrl, 0, IPMZ_PANEL_CTRL_WORDS * 4));
  Timer t;
  if (argc > 2 && std::string(argv[2]) == "probe") {  // f64 MFMA throughput vs independent chains, 1 WG per CU
    for (int threads : {256, 512})
      for (int nacc : {1, 2, 4, 8, 16}) {
        const int iters = 4000, blocks = 256;
        CK(ipmz::mfma_probe(D, blocks, 10, threads, nacc, st));
        t.start(st);
        CK(ipmz::mfma_probe(D, blocks, iters, threads, nacc, st));
        const float ms = t.stop(st);
        const double n_per_simd = (double)(threads / 64) / 4 * iters * nacc;
        std::printf("probe threads=%d nacc=%d: %.1f ns per MFMA per SIMD (%.2f TFLOP/s chip)\n", threads, nacc,
                    ms * 1e6 / n_per_simd, (double)blocks * (threads / 64) * iters * nacc * 2048.0 / ms / 1e9);
      }
    return 0;
  }
  if (argc > 2 && std::string(argv[2]) == "small") {  // batched one-workgroup factor (C4)
    for (int B : {1, 128, 256, 1024}) {
      double *Kb, *Db, *Lb, *Wb;
      const int64_t sK = ld * N, sL = (int64_t)((N + 63) / 64) * 64 * 64;
      CK(hipMalloc(&Kb, sK * B * 8));
      CK(hipMalloc(&Db, (int64_t)N * B * 8));
      CK(hipMalloc(&Lb, sL * B * 8));
      CK(hipMalloc(&Wb, (int64_t)N * 64 * B * 8));
      ipmz::BatchStrides bs;
      bs.B = B;
      bs.sK = sK;
      bs.sD = N;
      bs.sL = sL;
      bs.sW = (int64_t)N * 64;
      for (int q = 0; q < B; ++q) hipLaunchKernelGGL(fill_qd, dim3(64), dim3(256), 0, st, Kb + q * sK, ld, N, 7ull + q);
      unsigned long long clk[64];
      CK(ipmz::small_clock_probe(Kb, ld, N, Db, Lb, Wb, info, st, bs, clk));
      CK(hipStreamSynchronize(st));
      if (B == 1) {
        std::printf("small N=%d stage clocks (diag / trsm / update per block):", N);
        for (unsigned i = 1; i < clk[63] && i < 63; ++i) std::printf(" %llu", clk[i] - clk[i - 1]);
        std::printf("  total %llu\n", clk[clk[63] - 1] - clk[0]);
      }
      for (int q = 0; q < B; ++q) hipLaunchKernelGGL(fill_qd, dim3(64), dim3(256), 0, st, Kb + q * sK, ld, N, 7ull + q);
      t.start(st);
      CK(ipmz::ldlt_factor_small_batched(Kb, ld, N, Db, Lb, Wb, info, st, bs));
      std::printf("small factor N=%d B=%d: %.1f us\n", N, B, t.stop(st) * 1e3);
      CK(hipFree(Kb));
      CK(hipFree(Db));
      CK(hipFree(Lb));
      CK(hipFree(Wb));
    }
    return 0;
  }
  if (argc > 3 && std::string(argv[2]) == "gvar") {  // trailing-GEMM variants: kbench N gvar v1 v2 ...
    hipLaunchKernelGGL(fill_qd, dim3(2048), dim3(256), 0, st, K, ld, N, 7ull);
    for (int a = 3; a < argc; ++a) {
      const int var = std::atoi(argv[a]);
      if (var >= 20) {  // strip: M rows x 384 columns, rank 384
        for (int M : {3072, 6144, 8192, 10496}) {
          CK(ipmz::gemm_nt_sub_variant(var, M, 384, 384, W, 384, K, ld, K + 384 * ld + 384, ld, st));
          t.start(st);
          for (int r = 0; r < 10; ++r)
            CK(ipmz::gemm_nt_sub_variant(var, M, 384, 384, W, 384, K, ld, K + 384 * ld + 384, ld, st));
          const float us = t.stop(st) / 10 * 1e3;
          std::printf("gvar %2d strip M=%5d x 384 rank=384: %.1f us %.2f TFLOP/s\n", var, M, us,
                      2.0 * M * 384 * 384 / us / 1e6);
        }
        continue;
      }
      for (int rank : {256, 384})
        for (int R : {5632, N - rank}) {
          CK(ipmz::gemm_nt_sub_variant(var, R, R, rank, W, rank, K, ld, K + (int64_t)rank * ld + rank, ld, st));
          t.start(st);
          for (int r = 0; r < 5; ++r)
            CK(ipmz::gemm_nt_sub_variant(var, R, R, rank, W, rank, K, ld, K + (int64_t)rank * ld + rank, ld, st));
          const float ms = t.stop(st) / 5;
          std::printf("gvar %2d R=%5d rank=%d: %.3f ms %.2f TFLOP/s\n", var, R, rank, ms,
                      (double)R * (R + 1) * rank / ms / 1e9);
        }
    }
    return 0;
  }
  if (argc > 2 && std::string(argv[2]) == "gemm") {  // trailing GEMM alone (PMC passes)
    hipLaunchKernelGGL(fill_qd, dim3(2048), dim3(256), 0, st, K, ld, N, 7ull);
    const int R = N - 256;
    for (int r = 0; r < 3; ++r) {
      t.start(st);
      CK(ipmz::gemm_nt_sub(R, R, 256, W, 256, K, ld, K + 256 * ld + 256, ld, 0, 0, true, st));
      const float ms = t.stop(st);
      std::printf("trailing R=%d nbo=256: %.3f ms %.2f TFLOP/s\n", R, ms, (double)R * (R + 1) * 256 / ms / 1e9);
    }
    for (int M : {1024, 2048, 4096, 8192}) {  // look-ahead strip: M x 256, rank 256
      for (int var : {20, 21, 22}) {
        CK(ipmz::gemm_nt_sub_variant(var, M, 256, 256, W, 256, K, ld, K + 256 * ld + 256, ld, st));
        t.start(st);
        for (int r = 0; r < 10; ++r) CK(ipmz::gemm_nt_sub_variant(var, M, 256, 256, W, 256, K, ld, K + 256 * ld + 256, ld, st));
        std::printf("strip variant %d M=%d: %.1f us\n", var, M, t.stop(st) / 10 * 1e3);
      }
    }
    for (int R : {768, 1536, 3072, 4608}) {  // small trailing updates
      for (int var : {14, 23}) {
        CK(ipmz::gemm_nt_sub_variant(var, R, R, 256, W, 256, K, ld, K + 256 * ld + 256, ld, st));
        t.start(st);
        for (int r = 0; r < 10; ++r) CK(ipmz::gemm_nt_sub_variant(var, R, R, 256, W, 256, K, ld, K + 256 * ld + 256, ld, st));
        const float ms = t.stop(st) / 10;
        std::printf("trailing variant %d R=%d: %.1f us %.2f TFLOP/s\n", var, R, ms * 1e3, (double)R * (R + 1) * 256 / ms / 1e9);
      }
    }
    for (int var : {2, 9, 10, 14}) {
      for (int R : {5632, 11008}) {
        hipLaunchKernelGGL(fill_qd, dim3(2048), dim3(256), 0, st, K, ld, N, 7ull);
        CK(ipmz::gemm_nt_sub_variant(var, R, R, 256, W, 256, K, ld, K + 256 * ld + 256, ld, st));
        t.start(st);
        for (int r = 0; r < 5; ++r) CK(ipmz::gemm_nt_sub_variant(var, R, R, 256, W, 256, K, ld, K + 256 * ld + 256, ld, st));
        const float ms = t.stop(st) / 5;
        std::printf("gemm variant %d R=%d K=256: %.3f ms %.2f TFLOP/s\n", var, R, ms, (double)R * (R + 1) * 256 / ms / 1e9);
      }
    }
    return 0;
  }
  {  // panel-path pieces
    hipLaunchKernelGGL(fill_qd, dim3(2048), dim3(256), 0, st, K, ld, N, 7ull);
    for (int nbi : {64, -65, -69, 128}) {
      CK(ipmz::diag_probe(K, ld, 0, nbi, D, Linv, info, st));
      t.start(st);
      for (int r = 0; r < 10; ++r) CK(ipmz::diag_probe(K, ld, 1024 * r, nbi, D, Linv, info, st));
      std::printf("diag block nbi=%d: %.1f us\n", nbi, t.stop(st) / 10 * 1e3);
    }
    for (int j0 : {0, 5632, 10240}) {
      CK(ipmz::trsm_probe(K, ld, N, j0, D, Linv, W, 256, st));
      t.start(st);
      for (int r = 0; r < 10; ++r) CK(ipmz::trsm_probe(K, ld, N, j0, D, Linv, W, 256, st));
      std::printf("panel TRSM rows=%d x 64: %.1f us\n", N - j0 - 64, t.stop(st) / 10 * 1e3);
    }
    for (int cols : {64, 192, 256}) {
      for (int kd : {64, 256}) {
        const int M = N - 256;
        CK(ipmz::gemm_nt_sub(M, cols, kd, W, 256, K, ld, K + 256 * ld + 256, ld, 256, 256, false, st));
        t.start(st);
        for (int r = 0; r < 10; ++r)
          CK(ipmz::gemm_nt_sub(M, cols, kd, W, 256, K, ld, K + 256 * ld + 256, ld, 256, 256, false, st));
        const float us = t.stop(st) / 10 * 1e3;
        std::printf("strip update rows=%d cols=%d rank=%d: %.1f us (%.1f TFLOP/s)\n", M, cols, kd, us,
                    2.0 * M * cols * kd / us / 1e6);
      }
    }
  }
  {
    unsigned long long clk[32];
    for (int rep = 0; rep < 3; ++rep) {
      CK(ipmz::diag_clock_probe(K, ld, D, Linv, info, clk, st));
      CK(hipStreamSynchronize(st));
    }
    std::printf("diag64 blk stage clocks (s_memtime ticks from start):");
    for (unsigned i = 1; i < clk[31] && i < 31; ++i) std::printf(" %llu", clk[i] - clk[0]);
    std::printf("\n");
  }
  if (argc > 2 && std::string(argv[2]) == "pieces") return 0;
  for (int threads : {256}) {  // 0. f64 MFMA peak probe
    for (int nacc : {16}) {
      const int iters = 20000, blocks = 2048;
      CK(ipmz::mfma_probe(D, blocks, 10, threads, nacc, st));
      t.start(st);
      CK(ipmz::mfma_probe(D, blocks, iters, threads, nacc, st));
      const float ms = t.stop(st);
      const double fl = (double)blocks * (threads / 64) * iters * nacc * 2048.0;
      std::printf("mfma_f64_16x16x4 probe: threads=%d nacc=%d: %.2f TFLOP/s\n", threads, nacc, fl / ms / 1e9);
    }
  }
  for (int var = 2; var < 3; ++var) {
    for (int R : {5632, 11008}) {
      hipLaunchKernelGGL(fill_qd, dim3(2048), dim3(256), 0, st, K, ld, N, 7ull);
      CK(ipmz::gemm_nt_sub_variant(var, R, R, 256, W, 256, K, ld, K + 256 * ld + 256, ld, st));
      t.start(st);
      for (int r = 0; r < 5; ++r) CK(ipmz::gemm_nt_sub_variant(var, R, R, 256, W, 256, K, ld, K + 256 * ld + 256, ld, st));
      const float ms = t.stop(st) / 5;
      std::printf("gemm variant %d R=%d K=256: %.3f ms %.2f TFLOP/s\n", var, R, ms, (double)R * (R + 1) * 256 / ms / 1e9);
    }
  }
  // 1. trailing GEMM alone: rank-nbo update of an R x R lower region
  for (int nbo : {256}) {
    for (int R : {2048, 5632, 11008}) {
      if (R + nbo > N) continue;
      hipLaunchKernelGGL(fill_qd, dim3(2048), dim3(256), 0, st, K, ld, N, 7ull);
      CK(ipmz::gemm_nt_sub(R, R, nbo, W, nbo, K, ld, K + (int64_t)nbo * ld + nbo, ld, 0, 0, true, st));
      t.start(st);
      const int reps = 5;
      for (int r = 0; r < reps; ++r)
        CK(ipmz::gemm_nt_sub(R, R, nbo, W, nbo, K, ld, K + (int64_t)nbo * ld + nbo, ld, 0, 0, true, st));
      const float ms = t.stop(st) / reps;
      const double fl = (double)R * (R + 1) * nbo;
      std::printf("trailing nbo=%d R=%d: %.3f ms  %.2f TFLOP/s (algorithmic)\n", nbo, R, ms, fl / ms / 1e9);
    }
  }
  // 2. look-ahead factor: panel path on a high-priority stream, trailing
  // updates on a stream whose CU mask leaves `reserve` CUs to the panel path
  // (excl: the panel stream is confined to those CUs)
  std::vector<hipEvent_t> ev(2 * (N / 64 + 2) + 8);
  for (size_t i = 0; i < ev.size(); ++i) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  struct LA { int nbo, reserve; bool excl, fused; };
  const LA las[] = {{256, 0, false, false}, {256, 0, false, true}, {256, 32, false, true},
                    {512, 0, false, false}, {512, 0, false, true}, {512, 32, false, true}};
  for (const LA& la : las) {
    std::vector<uint32_t> mB((ncu + 31) / 32, 0u), mA((ncu + 31) / 32, 0u);
    const int stride = la.reserve ? ncu / la.reserve : ncu + 1;
    for (int c = 0; c < ncu; ++c) {
      const bool res = la.reserve && c % stride == 0 && c / stride < la.reserve;
      (res ? mA : mB)[c / 32] |= 1u << (c % 32);
    }
    hipStream_t sA, sB;
    CK(hipStreamCreateWithPriority(&sA, hipStreamNonBlocking, hi));
    if (la.reserve) CK(hipExtStreamCreateWithCUMask(&sB, (uint32_t)mB.size(), mB.data()));
    else CK(hipStreamCreateWithPriority(&sB, hipStreamNonBlocking, lo));
    if (la.excl) {
      CK(hipStreamDestroy(sA));
      CK(hipExtStreamCreateWithCUMask(&sA, (uint32_t)mA.size(), mA.data()));
    }
    {
      std::vector<uint32_t> got(mB.size(), 0u);
      CK(hipExtStreamGetCUMask(sB, (uint32_t)got.size(), got.data()));
      std::printf("config nbo=%d reserve=%d excl=%d: sB mask[0]=%08x\n", la.nbo, la.reserve, (int)la.excl, got[0]);
    }
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(fill_qd, dim3(2048), dim3(256), 0, sA, K, ld, N, 7ull);
      CK(hipStreamSynchronize(sA));
      t.start(sA);
      CK(ipmz::ldlt_factor(K, ld, N, D, Linv, W, la.nbo, 64, info, sA, nullptr, sB, ev.data(), (int)ev.size(),
                           la.fused ? pctrl : nullptr));
      const float fms = t.stop(sA);
      if (rep)
        std::printf("look-ahead factor N=%d nbo=%d reserve=%d%s%s: %.3f ms = %.2f TFLOP/s (N^3/3)\n", N, la.nbo,
                    la.reserve, la.excl ? " excl" : "", la.fused ? " fused" : "", fms,
                    (double)N * N * N / 3.0 / fms / 1e9);
    }
    CK(hipStreamSynchronize(sB));
    {
      unsigned hc[IPMZ_PANEL_CTRL_WORDS];
      CK(hipMemcpy(hc, pctrl, sizeof(hc), hipMemcpyDeviceToHost));
      std::printf("  panel ctrl: ticket=%u done=%u err=%u diag=%u\n", hc[0], hc[1], hc[2], hc[3]);
    }
    CK(hipStreamDestroy(sA));
    CK(hipStreamDestroy(sB));
  }
  const int cfg[][2] = {{256, 64}, {512, 64}, {128, 64}};
  for (auto& c : cfg) {
    hipLaunchKernelGGL(fill_qd, dim3(2048), dim3(256), 0, st, K, ld, N, 7ull);
    CK(hipMemsetAsync(info, 0x7f, 4, st));
    CK(ipmz::ldlt_factor(K, ld, N, D, Linv, W, c[0], c[1], info, st, nullptr, nullptr, nullptr, 0, pctrl));  // warm
    hipLaunchKernelGGL(fill_qd, dim3(2048), dim3(256), 0, st, K, ld, N, 7ull);
    t.start(st);
    CK(ipmz::ldlt_factor(K, ld, N, D, Linv, W, c[0], c[1], info, st, nullptr, nullptr, nullptr, 0, pctrl));
    const float fms = t.stop(st);
    {
      unsigned hc[IPMZ_PANEL_CTRL_WORDS];
      CK(hipMemcpy(hc, pctrl, sizeof(hc), hipMemcpyDeviceToHost));
      std::printf("  panel ctrl after factor: ticket=%u done=%u err=%u diag=%u\n", hc[0], hc[1], hc[2], hc[3]);
    }
    CK(hipMemsetAsync(b, 0, N * 8, st));
    t.start(st);
    for (int r = 0; r < 5; ++r) CK(ipmz::ldlt_solve(K, ld, N, D, Linv, c[1], b, side, st));
    float sms = t.stop(st) / 5;
    if (c[1] == 64) {
      t.start(st);
      for (int r = 0; r < 5; ++r) CK(ipmz::ldlt_solve_persistent(K, ld, N, D, Linv, 64, b, yb, zb, ctrl, st));
      const float pms = t.stop(st) / 5;
      std::printf("  persistent solve: %.3f ms (block-step chain %.3f ms)\n", pms, sms);
      sms = pms;
    }
    std::printf("factor N=%d nbo=%d nbi=%d: %.3f ms = %.2f TFLOP/s (N^3/3); solve %.3f ms\n", N, c[0], c[1], fms,
                (double)N * N * N / 3.0 / fms / 1e9, sms);
  }
  std::printf("done\n");
  return 0;
}
