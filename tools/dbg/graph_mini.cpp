// Minimal capture patterns, to find which construct the HIP runtime torch
// bundles (ROCm 7.0) cannot end a capture on (tools/dbg/repro_torch.py mini).
//   mini(which): 0 fork/join one side stream; 1 two side streams;
//   2 ping-pong (A waits B's event after B waited A's); 3 a side stream waits
//   an event recorded on another side stream; 4 an event recorded twice in
//   one capture; 5 a redundant wait (the dependency already reached through
//   another path); 6 two consecutive waits on one stream before a launch;
//   7 an event recorded on a stream with no node since its last wait.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::printf("%d %s -> %s\n", __LINE__, #x, hipGetErrorString(e_));           \
      return 2;                                                                    \
    }                                                                              \
  } while (0)

__global__ void tick(unsigned* p, unsigned v) {
  if (threadIdx.x == 0) atomicAdd(p, v);
}

extern "C" int mini(int which) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  hipStream_t o, a, b;
  CK(hipStreamCreateWithFlags(&o, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t e[8];
  for (auto& x : e) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
  unsigned* p;
  CK(hipMalloc(&p, 4));
  CK(hipMemset(p, 0, 4));
  auto K = [&](hipStream_t s, unsigned v) { hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, s, p, v); };
  CK(hipStreamBeginCapture(o, hipStreamCaptureModeThreadLocal));
  K(o, 1);
  CK(hipEventRecord(e[0], o));
  CK(hipStreamWaitEvent(a, e[0], 0));
  K(a, 10);
  if (which == 1 || which == 2 || which == 3 || which == 5 || which == 6) {
    CK(hipStreamWaitEvent(b, e[0], 0));
    K(b, 100);
  }
  if (which == 2) {  // ping-pong: b waits a, then a waits b
    CK(hipEventRecord(e[1], a));
    CK(hipStreamWaitEvent(b, e[1], 0));
    K(b, 1000);
    CK(hipEventRecord(e[2], b));
    CK(hipStreamWaitEvent(a, e[2], 0));
    K(a, 10000);
  }
  if (which == 3) {  // b waits an event recorded on a
    CK(hipEventRecord(e[1], a));
    CK(hipStreamWaitEvent(b, e[1], 0));
    K(b, 1000);
  }
  if (which == 4) {  // e[1] recorded twice
    CK(hipEventRecord(e[1], a));
    K(a, 1000);
    CK(hipEventRecord(e[1], a));
  }
  if (which == 5) {  // a waits b's event, which already depends on a's first node through o? (b waited e[0] only) + again a's own
    CK(hipEventRecord(e[1], a));
    CK(hipStreamWaitEvent(b, e[1], 0));
    CK(hipEventRecord(e[2], b));
    CK(hipStreamWaitEvent(a, e[2], 0));  // a's own node reached through b
    K(a, 1000);
  }
  if (which == 6) {  // two waits, then a launch
    CK(hipEventRecord(e[1], b));
    CK(hipEventRecord(e[2], o));
    CK(hipStreamWaitEvent(a, e[1], 0));
    CK(hipStreamWaitEvent(a, e[2], 0));
    K(a, 1000);
  }
  if (which == 7) {  // record on a right after a wait, no node in between
    CK(hipStreamWaitEvent(b, e[0], 0));
    CK(hipEventRecord(e[1], b));
    CK(hipStreamWaitEvent(a, e[1], 0));
    K(a, 1000);
  }
  // join every side stream back into o
  CK(hipEventRecord(e[6], a));
  CK(hipStreamWaitEvent(o, e[6], 0));
  if (which == 1 || which == 2 || which == 3 || which == 5 || which == 6 || which == 7) {
    CK(hipEventRecord(e[7], b));
    CK(hipStreamWaitEvent(o, e[7], 0));
  }
  K(o, 2);
  std::printf("mini %d: ending capture\n", which);
  hipGraph_t g;
  CK(hipStreamEndCapture(o, &g));
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, o));
  CK(hipStreamSynchronize(o));
  unsigned h;
  CK(hipMemcpy(&h, p, 4, hipMemcpyDeviceToHost));
  std::printf("mini %d ok sum %u\n", which, h);
  return 0;
}
