// The kbench "capture" experiment as a shared library, so that it runs on the
// HIP runtime of the process that loads it (torch bundles its own ROCm 7.0
// libamdhip64; the library and kbench are linked against /opt/rocm's 7.2).
//   python: import torch; torch.zeros(1, device="cuda"); ctypes.CDLL(".../libcapture_probe.so").capture_probe(N, NBO, DBG)
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
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

extern "C" int capture_probe(int N, int nbo_arg, int dbg_arg) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const int64_t ld = (N + 63) / 64 * 64;
  double *K, *D, *Linv, *W;
  int* info;
  unsigned* pctrl;
  CK(hipMalloc(&K, ld * N * 8));
  CK(hipMemset(K, 0, ld * N * 8));
  CK(hipMalloc(&D, N * 8));
  CK(hipMalloc(&Linv, (int64_t)(N + 127) / 64 * 128 * 128 * 8));
  CK(hipMalloc(&W, 3ll * N * 512 * 8));
  CK(hipMalloc(&info, 64));
  CK(hipMalloc(&pctrl, ipmz::panel_ctrl_words(N, 64) * 4));
    const int nbo = nbo_arg, dbg = dbg_arg;
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
    auto enqueue = [&]() -> int {  // capi.cpp factor_impl's sequence
      CK(hipMemsetAsync(info, 0x7f, 4, orig));
      CK(hipMemsetAsync(pctrl, 0, ipmz::panel_ctrl_words(N, nbo) * 4, orig));
      CK(hipEventRecord(ev[nev - 2], orig));
      CK(hipStreamWaitEvent(sA, ev[nev - 2], 0));
      CK(hipStreamWaitEvent(sB, ev[nev - 2], 0));
      CK(hipStreamWaitEvent(sC, ev[nev - 2], 0));
      CK(ipmz::ldlt_factor(K, ld, N, D, Linv, W, nbo, 64, info, sA, nullptr, sB, sC, ev.data(), nev - 2, pctrl));
      CK(hipEventRecord(ev[nev - 1], sA));
      CK(hipStreamWaitEvent(orig, ev[nev - 1], 0));
      return 0;
    };
    if (enqueue()) return 1;
    CK(hipStreamSynchronize(orig));
    std::printf("eager factor done (N=%d nbo=%d npan=%d)\n", N, nbo, npan);
    CK(hipStreamBeginCapture(orig, hipStreamCaptureModeThreadLocal));
    if (enqueue()) return 1;
    std::printf("enqueued, ending capture\n");
    hipGraph_t g = nullptr;
    CK(hipStreamEndCapture(orig, &g));
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    std::printf("captured: %zu nodes\n", nn);
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, orig));
    CK(hipStreamSynchronize(orig));
    unsigned hc[IPMZ_PANEL_CTRL_WORDS];
    CK(hipMemcpy(hc, pctrl, sizeof(hc), hipMemcpyDeviceToHost));
    std::printf("replayed ok%s\n", hc[ipmz::PANEL_ERR_WORD] ? " PANEL ERROR" : "");
    return 0;
}
