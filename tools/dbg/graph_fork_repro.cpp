// Stand-alone reproduction of the look-ahead factor's stream/event pattern
// under hipStreamBeginCapture (capi.cpp factor_impl + ldlt.hip ldlt_factor_t),
// with trivial kernels in place of the panel / GEMM launches.
//   graph_fork_repro NPAN VARIANT
// VARIANT bits:
//   1  streams without priorities
//   2  a fresh event for every record (no event recorded twice in a capture)
//   4  no evEntry (the caller-stream fork event only)
//   8  no third stream (rows launches on A)
//  16  eager run of the same pattern before the capture (what the product does)
//  32  two kernel launches per panel on A/C (the chain + rows launch pair)
//  64  a kernel and the factor's memsets (4 B, ctrl words, two vectors) on the caller's stream before the fork
// 128  a kernel on the caller's stream after the join
// 256  the product's launch conditions: no B / C launches past the last panels (p2, p3 >= N), no rows launch for the last panel
// Prints "ok" with the replayed result, or crashes / reports the error.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      std::printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      std::exit(2);                                                                       \
    }                                                                                     \
  } while (0)

__global__ void bump(unsigned* p, unsigned v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd(p, v);
}

struct Pool {
  std::vector<hipEvent_t> ev;
  bool fresh;
  size_t next = 0;
  hipEvent_t get(size_t i) {
    if (!fresh) {
      while (ev.size() <= i) {
        hipEvent_t e;
        CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ev.push_back(e);
      }
      return ev[i];
    }
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ev.push_back(e);
    return e;
  }
};

// the factor's fork / join, npan outer panels
static void pattern(Pool& pool, hipStream_t orig, hipStream_t sA, hipStream_t sB, hipStream_t sC, unsigned* p, int npan,
                    int var, char* scratch) {
  if (var & 64) {
    hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, orig, p, 7u);
    CK(hipMemsetAsync(scratch, 0x7f, 4, orig));
    CK(hipMemsetAsync(scratch + 256, 0, 4 * 1024 * 4, orig));
    CK(hipMemsetAsync(scratch + 65536, 0, 64, orig));
    CK(hipMemsetAsync(scratch + 131072, 0xff, 11264 * 8, orig));
    CK(hipMemsetAsync(scratch + 262144, 0xff, 11264 * 8, orig));
  }
  std::vector<hipEvent_t> evP(npan), evN(npan), evC(npan), evA(npan);
  // with reuse: the product's fixed slots; fresh: one event per record
  auto slot = [&](int base, int k) { return pool.get((size_t)base * npan + k); };
  const bool noC = var & 8;
  hipStream_t C = noC ? sA : sC;
  hipEvent_t fork = pool.get(4 * npan + 2);
  CK(hipEventRecord(fork, orig));
  CK(hipStreamWaitEvent(sA, fork, 0));
  CK(hipStreamWaitEvent(sB, fork, 0));
  if (!noC) CK(hipStreamWaitEvent(sC, fork, 0));
  if (!(var & 4)) {
    hipEvent_t entry = pool.get(4 * npan + 1);
    CK(hipEventRecord(entry, sA));
    CK(hipStreamWaitEvent(sB, entry, 0));
    if (!noC) CK(hipStreamWaitEvent(C, entry, 0));
  }
  const bool real = var & 256;
  auto panel = [&](int k) {
    hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, sA, p, 1u + k);
    if ((var & 32) && (!real || k + 1 < npan)) hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, C, p, 1000u + k);
  };
  panel(0);
  evA[0] = slot(3, 0);
  CK(hipEventRecord(evA[0], sA));
  evC[0] = slot(2, 0);
  CK(hipEventRecord(evC[0], C));
  CK(hipStreamWaitEvent(sA, evC[0], 0));
  for (int k = 0; k + 1 < npan; ++k) {
    evP[k] = slot(0, k);
    CK(hipEventRecord(evP[k], sA));
    CK(hipStreamWaitEvent(sB, evP[k], 0));
    if (!real || k + 2 < npan) hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, sB, p, 100000u);  // P_{k+2} columns
    evN[k] = slot(1, k);
    CK(hipEventRecord(evN[k], sB));
    if (!real || k + 3 < npan) hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, sB, p, 200000u);  // the trailing update
    if (k >= 1) {
      CK(hipStreamWaitEvent(sA, evN[k - 1], 0));
      if (!noC) CK(hipStreamWaitEvent(C, evN[k - 1], 0));
    }
    CK(hipStreamWaitEvent(C, evA[k], 0));
    if (!real || k + 2 < npan) hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, C, p, 300000u);  // the strip
    panel(k + 1);
    evA[k + 1] = slot(3, k + 1);
    CK(hipEventRecord(evA[k + 1], sA));
    evC[k + 1] = slot(2, k + 1);
    CK(hipEventRecord(evC[k + 1], C));
    CK(hipStreamWaitEvent(sA, evC[k + 1], 0));
  }
  hipEvent_t join = pool.get(4 * npan);
  CK(hipEventRecord(join, sB));
  CK(hipStreamWaitEvent(sA, join, 0));
  hipEvent_t j2 = pool.get(4 * npan + 3);
  CK(hipEventRecord(j2, sA));
  CK(hipStreamWaitEvent(orig, j2, 0));
  if (var & 128) hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, orig, p, 9u);
}

// as a shared library (-DREPRO_LIB): repro(npan, variant) on the HIP runtime of the loading process
#ifdef REPRO_LIB
extern "C" int repro(int npan, int var) {
#else
int main(int argc, char** argv) {
  const int npan = argc > 1 ? std::atoi(argv[1]) : 3;
  const int var = argc > 2 ? std::atoi(argv[2]) : 0;
#endif
  std::printf("npan %d variant %d\n", npan, var);
  std::fflush(stdout);
  hipStream_t orig, sA, sB, sC;
  CK(hipStreamCreateWithFlags(&orig, hipStreamNonBlocking));
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  if (var & 1) {
    CK(hipStreamCreateWithFlags(&sA, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sB, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sC, hipStreamNonBlocking));
  } else {
    CK(hipStreamCreateWithPriority(&sA, hipStreamNonBlocking, hi));
    CK(hipStreamCreateWithPriority(&sB, hipStreamNonBlocking, lo));
    CK(hipStreamCreateWithPriority(&sC, hipStreamNonBlocking, hi));
  }
  unsigned* p;
  CK(hipMalloc(&p, 4));
  CK(hipMemset(p, 0, 4));
  char* scratch;
  CK(hipMalloc(&scratch, 1 << 20));
  Pool pool{{}, (var & 2) != 0};  // shared by the eager run and the capture (the product's ctx pool)
  if (var & 16) {
    pattern(pool, orig, sA, sB, sC, p, npan, var, scratch);
    CK(hipStreamSynchronize(orig));
    std::printf("eager done\n");
    std::fflush(stdout);
  }
  CK(hipStreamBeginCapture(orig, hipStreamCaptureModeThreadLocal));
  pattern(pool, orig, sA, sB, sC, p, npan, var, scratch);
  std::printf("enqueued, ending capture\n");
  std::fflush(stdout);
  hipGraph_t g = nullptr;
  CK(hipStreamEndCapture(orig, &g));
  std::printf("captured\n");
  std::fflush(stdout);
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipMemset(p, 0, 4));
  CK(hipGraphLaunch(ge, orig));
  CK(hipStreamSynchronize(orig));
  unsigned h = 0;
  CK(hipMemcpy(&h, p, 4, hipMemcpyDeviceToHost));
  std::printf("ok: %zu nodes, sum %u\n", nn, h);
  return 0;
}
