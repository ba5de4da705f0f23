// Kernel micro-benchmark for libipmz (MI355X): times the factor pieces with
// HIP events.  Build: make -C ipm-zoo_amd kbench ; run:
//   ipm-zoo_amd/build/kbench N [factor|gemm|gvar v1 v2 ..|small|probe|diagclk]
// The experiment kernels (tile variants, probes) live in tools/kbench_probes.hip,
// outside the product library.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "kbench_probes.h"
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

__global__ void kb_to_f32(const double* __restrict__ s, float* __restrict__ d, int64_t n) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) d[i] = (float)s[i];
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
  const std::string mode = argc > 2 ? argv[2] : "factor";
  if (const char* dbg = std::getenv("KB_DEBUG")) ipmz::set_debug_inject_mask(std::atoi(dbg));  // tool only (A/B bits)
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const int64_t ld = (N + 63) / 64 * 64;
  double *K, *D, *Linv, *W, *b;
  int* info;
  CK(hipMalloc(&K, ld * N * 8));
  CK(hipMalloc(&D, N * 8));
  CK(hipMalloc(&Linv, (int64_t)(N + 127) / 64 * 128 * 128 * 8));
  CK(hipMalloc(&W, 3ll * N * 512 * 8));
  CK(hipMalloc(&b, N * 8));
  CK(hipMalloc(&info, 64));
  double *yb, *xb;
  unsigned *ctrl, *pctrl;
  CK(hipMalloc(&yb, N * 8));
  CK(hipMalloc(&xb, N * 8));
  CK(hipMalloc(&ctrl, 256));
  CK(hipMemset(ctrl, 0, 256));
  CK(hipMalloc(&pctrl, ipmz::panel_ctrl_words(N, 64) * 4));
  CK(hipMemset(pctrl, 0, ipmz::panel_ctrl_words(N, 64) * 4));
  Timer t;
  hipLaunchKernelGGL(fill_qd, dim3(2048), dim3(256), 0, st, K, ld, N, 7ull);
  if (mode == "solvecmp") {  // kbench_stamps N solvecmp: the persistent solve in fp64 and fp32 on one factor
    hipStream_t sB, sC;
    CK(hipStreamCreate(&sB));
    CK(hipStreamCreate(&sC));
    std::vector<hipEvent_t> ev(3 * (N / 64 + 2) + 8);
    for (size_t i = 0; i < ev.size(); ++i) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    CK(ipmz::ldlt_factor(K, ld, N, D, Linv, W, 512, 64, info, st, nullptr, sB, sC, ev.data(), (int)ev.size(), pctrl));
    CK(hipStreamSynchronize(st));
    CK(hipDeviceSynchronize());
    const int nb = (N + 127) / 128;
    static unsigned long long stp[2][256][6];
    auto report = [&](const char* tag, float ms) {
      CK(ipmz::solve_stamps(&stp[0][0][0]));
      double hop = 0, det = 0, post = 0, wait = 0;
      int late = 0, cnt = 0;
      for (int j = 4; j < nb && j < 256; ++j) {
        const double s1 = (double)stp[0][j - 1][3], s = (double)stp[0][j][3], seen = (double)stp[0][j][4],
                     cin = (double)stp[0][j][2];
        hop += s - s1, det += seen - s1, post += s - seen, wait += seen - cin;
        late += cin > s1;
        ++cnt;
      }
      std::printf("%s N=%d: %.3f ms per solve (2 sweeps); forward hops %d..%d: hop %.2f us = detect %.2f + post %.2f; "
                  "critical wait %.2f us; blocks whose bulk finished after y_{J-1}: %d\n",
                  tag, N, ms, 4, nb - 1, hop / cnt / 100.0, det / cnt / 100.0, post / cnt / 100.0, wait / cnt / 100.0,
                  late);
      // block J's clocks relative to the store of y_{J-1}
      double rel[5] = {0, 0, 0, 0, 0};
      for (int j = 4; j < nb && j < 256; ++j)
        for (int i = 0; i < 5; ++i) rel[i] += ((double)stp[0][j][i] - (double)stp[0][j - 1][3]) / 100.0;
      std::printf("   block J vs y_{J-1} stored (us): start %.2f, bulk done %.2f, at hand-off %.2f, "
                  "y_{J-1} seen %.2f, y_J stored %.2f; previous stores: y_{J-2} %.2f, y_{J-3} %.2f\n",
                  rel[0] / cnt, rel[1] / cnt, rel[2] / cnt, rel[4] / cnt, rel[3] / cnt, -hop / cnt / 100.0,
                  -2 * hop / cnt / 100.0);
    };
    double* P;
    CK(hipMalloc(&P, ipmz::solve_prep_elems(N) * 8));
    CK(hipMemsetAsync(b, 0, N * 8, st));
    CK(ipmz::solve_reset(yb, xb, 8, N, ctrl, st));
    CK(ipmz::solve_prep(K, ld, N, Linv, P, st));
    CK(ipmz::ldlt_solve_persistent(K, ld, N, D, P, b, yb, xb, ctrl, st));
    t.start(st);
    for (int r = 0; r < 5; ++r) CK(ipmz::ldlt_solve_persistent(K, ld, N, D, P, b, yb, xb, ctrl, st));
    report("fp64", t.stop(st) / 5);
    // the same factor in fp32
    float *K32, *D32, *L32, *P32, *b32, *y32, *x32;
    const int64_t nl = (int64_t)(N + 127) / 64 * 128 * 128;
    CK(hipMalloc(&K32, ld * N * 4));
    CK(hipMalloc(&D32, N * 4));
    CK(hipMalloc(&L32, nl * 4));
    CK(hipMalloc(&P32, ipmz::solve_prep_elems(N) * 4));
    CK(hipMalloc(&b32, N * 4));
    CK(hipMalloc(&y32, N * 4));
    CK(hipMalloc(&x32, N * 4));
    hipLaunchKernelGGL(kb_to_f32, dim3(2048), dim3(256), 0, st, K, K32, ld * N);
    hipLaunchKernelGGL(kb_to_f32, dim3(64), dim3(256), 0, st, D, D32, (int64_t)N);
    hipLaunchKernelGGL(kb_to_f32, dim3(512), dim3(256), 0, st, Linv, L32, nl);
    CK(hipMemsetAsync(b32, 0, N * 4, st));
    CK(ipmz::solve_reset(y32, x32, 4, N, ctrl, st));
    CK(ipmz::solve_prep(K32, ld, N, L32, P32, st));
    CK(ipmz::ldlt_solve_persistent(K32, ld, N, D32, P32, b32, y32, x32, ctrl, st));
    t.start(st);
    for (int r = 0; r < 5; ++r) CK(ipmz::ldlt_solve_persistent(K32, ld, N, D32, P32, b32, y32, x32, ctrl, st));
    report("fp32", t.stop(st) / 5);
    unsigned hctrl[8];
    CK(hipMemcpy(hctrl, ctrl, sizeof(hctrl), hipMemcpyDeviceToHost));
    std::printf("%s\ndone\n", hctrl[ipmz::SOLVE_ERR_WORD] ? "SOLVE ERROR" : "ok");
    return 0;
  }
  if (mode == "capture") {  // kbench N capture NBO DBG: the product factor's fork/join under hipStreamBeginCapture
    const int nbo = argc > 3 ? std::atoi(argv[3]) : 256;
    const int dbg = argc > 4 ? std::atoi(argv[4]) : 0;
    ipmz::set_debug_inject_mask(dbg);
    const int npan = (N + nbo - 1) / nbo, nev = 4 * npan + 4;
    std::vector<hipEvent_t> ev(nev);
    for (auto& evi : ev) CK(hipEventCreateWithFlags(&evi, hipEventDisableTiming));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t orig, sA, sB, sC;
    CK(hipStreamCreateWithFlags(&orig, hipStreamNonBlocking));
    CK(hipStreamCreateWithPriority(&sA, hipStreamNonBlocking, hi));
    CK(hipStreamCreateWithPriority(&sB, hipStreamNonBlocking, lo));
    CK(hipStreamCreateWithPriority(&sC, hipStreamNonBlocking, hi));
    CK(hipStreamSynchronize(st));
    auto enqueue = [&]() {  // capi.cpp factor_impl's sequence
      CK(hipMemsetAsync(info, 0x7f, 4, orig));
      CK(hipMemsetAsync(pctrl, 0, ipmz::panel_ctrl_words(N, nbo) * 4, orig));
      CK(hipEventRecord(ev[nev - 2], orig));
      CK(hipStreamWaitEvent(sA, ev[nev - 2], 0));
      CK(hipStreamWaitEvent(sB, ev[nev - 2], 0));
      CK(hipStreamWaitEvent(sC, ev[nev - 2], 0));
      CK(ipmz::ldlt_factor(K, ld, N, D, Linv, W, nbo, 64, info, sA, nullptr, sB, sC, ev.data(), nev - 2, pctrl));
      CK(hipEventRecord(ev[nev - 1], sA));
      CK(hipStreamWaitEvent(orig, ev[nev - 1], 0));
    };
    enqueue();
    CK(hipStreamSynchronize(orig));
    std::printf("eager factor done (N=%d nbo=%d npan=%d)\n", N, nbo, npan);
    CK(hipStreamBeginCapture(orig, hipStreamCaptureModeThreadLocal));
    enqueue();
    std::printf("enqueued, ending capture\n");
    hipGraph_t g = nullptr;
    CK(hipStreamEndCapture(orig, &g));
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    std::printf("captured: %zu nodes\n", nn);
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipLaunchKernelGGL(fill_qd, dim3(2048), dim3(256), 0, orig, K, ld, N, 7ull);
    CK(hipGraphLaunch(ge, orig));
    CK(hipStreamSynchronize(orig));
    unsigned hc[IPMZ_PANEL_CTRL_WORDS];
    CK(hipMemcpy(hc, pctrl, sizeof(hc), hipMemcpyDeviceToHost));
    std::printf("replayed ok%s\n", hc[ipmz::PANEL_ERR_WORD] ? " PANEL ERROR" : "");
    return 0;
  }
  if (mode == "probe") {  // f64 MFMA throughput vs independent chains, 1 WG per CU
    for (int threads : {256, 512})
      for (int nacc : {1, 4, 8, 16}) {
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
  if (mode == "diagclk") {  // stage clocks of the 64 x 64 diagonal factor; column passes 0 (as shipped), 1 (variant)
    std::vector<double> ref;
    for (int cpv : {9, 11, 12, 9, 11, 12, 9, 11, 12}) {  // kbench_probes.hip diag_clock_probe
      unsigned long long clk[32];
      for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(fill_qd, dim3(2048), dim3(256), 0, st, K, ld, N, 7ull);
        CK(ipmz::diag_clock_probe(K, ld, D, Linv, info, clk, st, cpv));
        CK(hipStreamSynchronize(st));
      }
      std::vector<double> hk(64 * ld), hd(64), hl(64 * 64);
      CK(hipMemcpy(hk.data(), K, 64 * ld * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hd.data(), D, 64 * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hl.data(), Linv, 64 * 64 * 8, hipMemcpyDeviceToHost));
      std::vector<double> cur(hd);
      for (int i = 0; i < 64; ++i)
        for (int j = 0; j < i; ++j) cur.push_back(hk[i * ld + j]);
      cur.insert(cur.end(), hl.begin(), hl.end());
      double dmax = 0;
      if (ref.empty()) ref = cur;
      else
        for (size_t i = 0; i < cur.size(); ++i) dmax = std::max(dmax, std::fabs(cur[i] - ref[i]));
      std::printf("diag64 v=%2d stage clocks (s_memtime ticks from start):", cpv);
      for (unsigned i = 1; i < clk[31] && i < 31; ++i) std::printf(" %llu", clk[i] - clk[0]);
      std::printf("  (max |d| vs the first: %.2e)\n", dmax);
    }
    return 0;
  }
  if (mode == "small") {  // batched one-workgroup factor (C4)
    for (int B : {128, 256, 1024}) {
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
      CK(ipmz::ldlt_factor_small_batched(Kb, ld, N, Db, Lb, Wb, info, st, bs));  // warm
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
  if (mode == "smallv") {  // kbench 320 smallv: the one-workgroup factors: right-looking (8 waves) vs left-looking
    std::vector<double> refK, refD;
    std::vector<int> vars = {8, 1};
    for (int a = 3; a < argc; ++a) vars.push_back(std::atoi(argv[a]));  // e.g. 101 102 104 (attribution)
    for (int B : {128, 1024})
      for (int snw : vars) {
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
        float best = 1e30f;
        for (int rep = 0; rep < 4; ++rep) {
          for (int q = 0; q < B; ++q) hipLaunchKernelGGL(fill_qd, dim3(64), dim3(256), 0, st, Kb + q * sK, ld, N, 7ull + q);
          t.start(st);
          CK(ipmz::ldlt_factor_small_variant(snw, Kb, ld, N, Db, Lb, Wb, info, st, bs));
          const float ms = t.stop(st);
          if (rep) best = ms < best ? ms : best;
        }
        std::vector<double> hD(N), hK(sK);
        CK(hipMemcpy(hD.data(), Db + (int64_t)(B - 1) * N, N * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hK.data(), Kb + (int64_t)(B - 1) * sK, sK * 8, hipMemcpyDeviceToHost));
        double cs = 0;
        for (double d : hD) cs += d;
        // the variants against the first (right-looking) one: D and the strict lower L
        double dD = 0, dL = 0;
        if (snw == 8) {
          refD = hD;
          refK = hK;
        } else {
          for (int i = 0; i < N; ++i) {
            dD = std::max(dD, std::fabs(hD[i] - refD[i]) / std::max(1.0, std::fabs(refD[i])));
            for (int j = 0; j < i; ++j) dL = std::max(dL, std::fabs(hK[i * ld + j] - refK[i * ld + j]));
          }
        }
        std::printf("small factor N=%d B=%d variant=%s: %.1f us (D checksum of the last QP %.15e; vs right-looking: "
                    "max rel dD %.2e, max dL %.2e)\n",
                    N, B, snw >= 100 ? ("left-exp" + std::to_string(snw - 100)).c_str() : snw == 2 ? "left-ws" : snw == 1 ? "left" : snw == 4 ? "right-4w" : "right",
                    best * 1e3, cs, dD, dL);
        CK(hipFree(Kb));
        CK(hipFree(Db));
        CK(hipFree(Lb));
        CK(hipFree(Wb));
      }
    return 0;
  }
  if (mode == "smalldet") {  // kbench 320 smalldet v1 v2 ...: run-to-run bitwise determinism of the small factors
    const int B = 1024, R = 40;
    for (int a = 3; a < argc; ++a) {
      const int snw = std::atoi(argv[a]);
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
      std::vector<double> rK(sK * B), rD((int64_t)N * B), hK(sK * B), hD((int64_t)N * B);
      int bad_runs = 0;
      for (int rep = 0; rep <= R; ++rep) {
        for (int q = 0; q < B; ++q) hipLaunchKernelGGL(fill_qd, dim3(64), dim3(256), 0, st, Kb + q * sK, ld, N, 7ull + q);
        CK(ipmz::ldlt_factor_small_variant(snw, Kb, ld, N, Db, Lb, Wb, info, st, bs));
        CK(hipStreamSynchronize(st));
        std::vector<double>& K_ = rep ? hK : rK;
        std::vector<double>& D_ = rep ? hD : rD;
        CK(hipMemcpy(K_.data(), Kb, sK * B * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(D_.data(), Db, (int64_t)N * B * 8, hipMemcpyDeviceToHost));
        if (!rep) continue;
        int badq = 0, first = -1, fi = -1, fj = -1;
        for (int q = 0; q < B; ++q) {
          bool bad = std::memcmp(&hD[(int64_t)q * N], &rD[(int64_t)q * N], N * 8) != 0;
          for (int i = 0; i < N && !bad; ++i)
            for (int j = 0; j < i; ++j)
              if (std::memcmp(&hK[q * sK + i * ld + j], &rK[q * sK + i * ld + j], 8)) {
                bad = true;
                if (first < 0) { fi = i; fj = j; }
                break;
              }
          if (bad) {
            ++badq;
            if (first < 0) first = q;
          }
        }
        if (badq) {
          ++bad_runs;
          std::printf("smalldet variant %d run %d: %d QPs differ (first QP %d, first L entry (%d,%d))\n", snw, rep, badq,
                      first, fi, fj);
        }
      }
      std::printf("smalldet variant %d: %d of %d runs differ bitwise from run 0\n", snw, bad_runs, R);
      CK(hipFree(Kb));
      CK(hipFree(Db));
      CK(hipFree(Lb));
      CK(hipFree(Wb));
    }
    return 0;
  }
  if (mode == "gvar") {  // trailing-GEMM tile variants: kbench N gvar v1 v2 ...
    for (int a = 3; a < argc; ++a) {
      const int var = std::atoi(argv[a]);
      if (var >= 20) {  // strip: M rows x 512 columns, rank 512 (the look-ahead strips at nbo = 512)
        for (int M : {3072, 6144, 8192, 10240}) {
          CK(ipmz::gemm_nt_sub_variant(var, M, 512, 512, W, 512, K, ld, K + 512 * ld + 512, ld, st));
          t.start(st);
          for (int r = 0; r < 10; ++r)
            CK(ipmz::gemm_nt_sub_variant(var, M, 512, 512, W, 512, K, ld, K + 512 * ld + 512, ld, st));
          const float us = t.stop(st) / 10 * 1e3;
          std::printf("gvar %2d strip M=%5d x 512 rank=512: %.1f us %.2f TFLOP/s\n", var, M, us,
                      2.0 * M * 512 * 512 / us / 1e6);
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
  if (mode == "g32") {  // fp32 trailing-update variants: kbench N g32 v1 v2 ... (rank 512, R = N - 512)
    float* K32 = reinterpret_cast<float*>(K);
    float* W32 = reinterpret_cast<float*>(W);
    const int64_t ld32 = ld;
    for (int a = 3; a < argc; ++a) {
      const int var = std::atoi(argv[a]);
      for (int R : {N / 2, N - 512}) {
        const int rank = 512;
        hipError_t e = ipmz::gemm_nt_sub_variant32(var, R, R, rank, W32, rank, K32, ld32, K32 + (int64_t)rank * ld32 + rank, ld32, st);
        if (e != hipSuccess) {
          std::printf("g32 %d: %s\n", var, hipGetErrorString(e));
          break;
        }
        t.start(st);
        for (int r = 0; r < 5; ++r)
          CK(ipmz::gemm_nt_sub_variant32(var, R, R, rank, W32, rank, K32, ld32, K32 + (int64_t)rank * ld32 + rank, ld32, st));
        const float ms = t.stop(st) / 5;
        std::printf("g32 %2d R=%5d rank=%d: %.3f ms %.2f TFLOP/s\n", var, R, rank, ms, (double)R * (R + 1) * rank / ms / 1e9);
      }
    }
    return 0;
  }
  if (mode == "sustain") {  // the trailing update back to back: clock / power drift over ~60 ms
    const int rank = 512, R = N - 3 * rank;
    for (int g = 0; g < 8; ++g) {
      t.start(st);
      for (int r = 0; r < 8; ++r)
        CK(ipmz::gemm_nt_sub(R, R, rank, W, rank, K, ld, K + (int64_t)rank * ld + rank, ld, 0, 0, true, st));
      const float ms = t.stop(st) / 8;
      std::printf("sustain group %d R=%d rank=%d: %.3f ms %.2f TFLOP/s\n", g, R, rank, ms,
                  (double)R * (R + 1) * rank / ms / 1e9);
    }
    return 0;
  }
  if (mode == "gemm") {  // the product's trailing update alone (PMC passes)
    for (int rank : {256, 384}) {
      const int R = N - rank;
      for (int r = 0; r < 3; ++r) {
        t.start(st);
        CK(ipmz::gemm_nt_sub(R, R, rank, W, rank, K, ld, K + (int64_t)rank * ld + rank, ld, 0, 0, true, st));
        const float ms = t.stop(st);
        std::printf("trailing R=%d rank=%d: %.3f ms %.2f TFLOP/s\n", R, rank, ms, (double)R * (R + 1) * rank / ms / 1e9);
      }
    }
    return 0;
  }
  if (mode == "chainclk") {  // kbench_chain N chainclk NBO: per-block clocks of the panel chain (IPMZ_CHAIN_STAMPS)
    const int nbo = argc > 3 ? std::atoi(argv[3]) : 512;
    std::vector<hipEvent_t> ev(5 * (N / 64 + 2) + 8);
    for (auto& evi : ev) CK(hipEventCreateWithFlags(&evi, hipEventDisableTiming));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t sA, sB, sC;
    const int rcu = std::getenv("KB_CUS") ? std::atoi(std::getenv("KB_CUS")) : 0;
    if (rcu > 0) {  // chain stream on the top rcu CUs, trailing stream on the rest
      hipDeviceProp_t pr;
      CK(hipGetDeviceProperties(&pr, 0));
      const int ncu = pr.multiProcessorCount;
      std::vector<uint32_t> ma((ncu + 31) / 32, 0u), mb((ncu + 31) / 32, 0u);
      for (int i = 0; i < ncu; ++i) (i >= ncu - rcu ? ma : mb)[i / 32] |= 1u << (i % 32);
      CK(hipExtStreamCreateWithCUMask(&sA, (uint32_t)ma.size(), ma.data()));
      CK(hipExtStreamCreateWithCUMask(&sB, (uint32_t)mb.size(), mb.data()));
      CK(hipExtStreamCreateWithCUMask(&sC, (uint32_t)mb.size(), mb.data()));
      std::printf("chain stream on %d of %d CUs, trailing and rows on the rest\n", rcu, ncu);
    } else {
      CK(hipStreamCreateWithPriority(&sA, hipStreamNonBlocking, hi));
      CK(hipStreamCreateWithPriority(&sB, hipStreamNonBlocking, lo));
      CK(hipStreamCreateWithPriority(&sC, hipStreamNonBlocking, hi));
    }
    static unsigned long long cs[IPMZ_CHAIN_STAMP_BLOCKS][16], hs[IPMZ_CHAIN_STAMP_BLOCKS][4];
    for (int rep = 0; rep < 4; ++rep) {
      hipLaunchKernelGGL(fill_qd, dim3(2048), dim3(256), 0, sA, K, ld, N, 7ull);
      CK(hipMemsetAsync(pctrl, 0, ipmz::panel_ctrl_words(N, nbo) * 4, sA));
      CK(hipStreamSynchronize(sA));
      t.start(sA);
      CK(hipEventRecord(ev.back(), sA));
      CK(hipStreamWaitEvent(sB, ev.back(), 0));
      CK(hipStreamWaitEvent(sC, ev.back(), 0));
      CK(ipmz::ldlt_factor(K, ld, N, D, Linv, W, nbo, 64, info, sA, nullptr, sB, sC, ev.data(), (int)ev.size() - 1,
                           pctrl));
      const float fms = t.stop(sA);
      CK(hipDeviceSynchronize());
      std::printf("factor N=%d nbo=%d: %.3f ms\n", N, nbo, fms);
    }
    CK(ipmz::chain_stamps(&cs[0][0], &hs[0][0]));
    const double t0 = (double)cs[0][0];
    auto us = [&](unsigned long long v) { return v ? (v - t0) / 100.0 : -1.0; };
    std::printf("block: diag_start ready_seen diag_done ops_loaded trsm_done own_done | helper_ready(blk) | "
                "rows0 start end | launch starts (us from block 0's diag start); dur = next diag start - this\n");
    const int nblk = (N + 63) / 64;
    for (int b = 0; b < nblk && b < IPMZ_CHAIN_STAMP_BLOCKS; ++b) {
      const double nx = b + 1 < nblk ? us(cs[b + 1][0]) : -1.0;
      std::printf("%3d %9.2f %9.2f %9.2f %9.2f %9.2f %9.2f | %9.2f | %9.2f %9.2f | %9.2f %9.2f | dur %6.2f", b,
                  us(cs[b][0]), us(cs[b][1]), us(cs[b][2]), us(cs[b][3]), us(cs[b][4]), us(cs[b][5]), us(hs[b][0]),
                  us(hs[b][1]), us(hs[b][2]), us(hs[b][3]), -1.0, nx > 0 ? nx - us(cs[b][0]) : 0.0);
      if (cs[b][6])  // rows role 0 at this block: DIAG seen, TRSM done, strips done
        std::printf(" | rows0 %9.2f %9.2f %9.2f", us(cs[b][6]), us(cs[b][7]), us(cs[b][8]));
      std::printf("\n");
    }
    return 0;
  }
  // factor: the look-ahead factor (panel path on a high-priority stream,
  // trailing updates on a low-priority one) and the persistent solve.
  // (Measured and dropped: CU masks reserving 8 / 16 / 32 CUs for the panel
  // streams, a persistent trailing-GEMM grid of 248-512 workgroups -- no gain;
  // the next-but-one panel's column update on a fourth stream beside the
  // trailing update: 12.22 -> 12.11 ms here, C3 72 -> 66 steps/s in the graph.)
  std::vector<hipEvent_t> ev(3 * (N / 64 + 2) + 8);
  for (size_t i = 0; i < ev.size(); ++i) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t sA, sB, sC;
  CK(hipStreamCreateWithPriority(&sA, hipStreamNonBlocking, hi));
  CK(hipStreamCreateWithPriority(&sB, hipStreamNonBlocking, lo));
  CK(hipStreamCreateWithPriority(&sC, hipStreamNonBlocking, hi));
  for (int a = 3; a < argc || a == 3; ++a) {
    const int nbo = argc > a ? std::atoi(argv[a]) : 384;
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(fill_qd, dim3(2048), dim3(256), 0, sA, K, ld, N, 7ull);
      CK(hipMemsetAsync(pctrl, 0, ipmz::panel_ctrl_words(N, 64) * 4, sA));
      CK(hipStreamSynchronize(sA));
      t.start(sA);
      CK(hipEventRecord(ev.back(), sA));
      CK(hipStreamWaitEvent(sB, ev.back(), 0));
      CK(hipStreamWaitEvent(sC, ev.back(), 0));
      CK(ipmz::ldlt_factor(K, ld, N, D, Linv, W, nbo, 64, info, sA, nullptr, sB, sC, ev.data(), (int)ev.size() - 1,
                           pctrl));
      const float fms = t.stop(sA);
      if (rep) best = fms < best ? fms : best;
    }
    CK(hipStreamSynchronize(sB));
    unsigned hc[IPMZ_PANEL_CTRL_WORDS];
    CK(hipMemcpy(hc, pctrl, sizeof(hc), hipMemcpyDeviceToHost));
    std::printf("look-ahead factor N=%d nbo=%d: %.3f ms = %.2f TFLOP/s%s\n", N, nbo, best,
                (double)N * N * N / 3.0 / best / 1e9, hc[ipmz::PANEL_ERR_WORD] ? " PANEL ERROR" : "");
  }
  CK(hipMemsetAsync(b, 0, N * 8, st));
  double* P;
  CK(hipMalloc(&P, ipmz::solve_prep_elems(N) * 8));
  CK(ipmz::solve_reset(yb, xb, 8, N, ctrl, st));
  t.start(st);
  CK(ipmz::solve_prep(K, ld, N, Linv, P, st));
  const float pms = t.stop(st);
  CK(ipmz::ldlt_solve_persistent(K, ld, N, D, P, b, yb, xb, ctrl, st));
  t.start(st);
  for (int r = 0; r < 5; ++r) CK(ipmz::ldlt_solve_persistent(K, ld, N, D, P, b, yb, xb, ctrl, st));
  const float sms = t.stop(st) / 5;
  {
    static unsigned long long stp[2][256][6];
    CK(ipmz::solve_stamps(&stp[0][0][0]));
    const double t0 = (double)stp[0][0][0];
    std::printf("fwd block: start bulkdone critin seen stored (us from block 0 start)\n");
    for (int j = 0; j < (N + 127) / 128 && j < 256; ++j)
      std::printf("%3d %8.2f %8.2f %8.2f %8.2f %8.2f\n", j, (stp[0][j][0] - t0) / 100.0, (stp[0][j][1] - t0) / 100.0,
                  (stp[0][j][2] - t0) / 100.0, (stp[0][j][4] - t0) / 100.0, (stp[0][j][3] - t0) / 100.0);
  }
  unsigned hctrl[8];
  CK(hipMemcpy(hctrl, ctrl, sizeof(hctrl), hipMemcpyDeviceToHost));
  std::printf("solve prep N=%d: %.3f ms%s\n", N, pms, hctrl[ipmz::SOLVE_ERR_WORD] ? " SOLVE ERROR" : "");
  std::printf("persistent solve N=%d: %.3f ms (%.2f TB/s over the 2 x N^2/2 x 8 B of L)\n", N, sms,
              8.0 * N * (double)N / sms / 1e9);
  std::printf("done\n");
  return 0;
}
