// Minimal capture patterns, to find which construct the HIP runtime torch
// bundles (ROCm 7.0) cannot end a capture on (tools/dbg/repro_torch.py mini).
//   mini(which): 0 fork/join one side stream; 1 two side streams;
//   2 ping-pong (A waits B's event after B waited A's); 3 a side stream waits
//   an event recorded on another side stream; 4 an event recorded twice in
//   one capture; 5 a redundant wait (the dependency already reached through
//   another path); 6 two consecutive waits on one stream before a launch;
//   7 an event recorded on a stream with no node since its last wait;
//   8, 9: 2 and 5 with the waits through wait_pruned (the dependency set of
//   the capturing stream reduced: duplicates and ancestors of other members dropped);
//   10, 11: 2 and 5 with cross-stream waits as explicit capture dependencies
//   (the event's nodes noted at record time, added to the waiter with
//   hipStreamUpdateCaptureDependencies: no hipStreamWaitEvent between side streams).
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

// is `a` an ancestor of `b` (or b itself) in the graph being captured?
static bool reaches(hipGraphNode_t a, hipGraphNode_t b, int depth = 0) {
  if (a == b) return true;
  if (depth > 4096) return false;
  size_t n = 0;
  if (hipGraphNodeGetDependencies(b, nullptr, &n) != hipSuccess || n == 0) return false;
  hipGraphNode_t deps[64];
  if (n > 64) n = 64;
  hipGraphNodeGetDependencies(b, deps, &n);
  for (size_t i = 0; i < n; ++i)
    if (reaches(a, deps[i], depth + 1)) return true;
  return false;
}
static hipError_t wait_pruned(hipStream_t s, hipEvent_t e) {
  hipError_t r = hipStreamWaitEvent(s, e, 0);
  if (r != hipSuccess) return r;
  hipStreamCaptureStatus cs;
  unsigned long long id;
  hipGraph_t g;
  const hipGraphNode_t* deps = nullptr;
  size_t n = 0;
  if ((r = hipStreamGetCaptureInfo_v2(s, &cs, &id, &g, &deps, &n)) != hipSuccess) return r;
  if (cs != hipStreamCaptureStatusActive || n < 2) return hipSuccess;
  hipGraphNode_t keep[64];
  size_t m = 0;
  for (size_t i = 0; i < n && i < 64; ++i) {
    bool drop = false;
    for (size_t j = 0; j < n && !drop; ++j)
      if (j != i && (deps[i] == deps[j] ? j < i : reaches(deps[i], deps[j]))) drop = true;
    if (!drop) keep[m++] = deps[i];
  }
  std::printf("  wait_pruned: %zu -> %zu dependencies\n", n, m);
  return hipStreamUpdateCaptureDependencies(s, keep, m, hipStreamSetCaptureDependencies);
}

static hipGraphNode_t g_nodes[8][16];
static size_t g_n[8];
static hipError_t rec_noted(hipEvent_t* e, int i, hipStream_t s) {
  hipError_t r = hipEventRecord(e[i], s);
  if (r != hipSuccess) return r;
  hipStreamCaptureStatus cs;
  unsigned long long id;
  hipGraph_t g;
  const hipGraphNode_t* deps = nullptr;
  size_t n = 0;
  if ((r = hipStreamGetCaptureInfo_v2(s, &cs, &id, &g, &deps, &n)) != hipSuccess) return r;
  g_n[i] = n;
  for (size_t k = 0; k < n && k < 16; ++k) g_nodes[i][k] = deps[k];
  return hipSuccess;
}
static hipError_t wait_noted(hipStream_t s, int i) {
  return hipStreamUpdateCaptureDependencies(s, g_nodes[i], g_n[i], hipStreamAddCaptureDependencies);
}

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
  const bool pr = which == 8 || which == 9, nt = which == 10 || which == 11;
  if (which == 8 || which == 10) which = 2;
  if (which == 9 || which == 11) which = 5;
  auto W = [&](hipStream_t s, hipEvent_t ev) {
    if (nt) return wait_noted(s, (int)(&ev - &ev) + (ev == e[1] ? 1 : 2));
    return pr ? wait_pruned(s, ev) : hipStreamWaitEvent(s, ev, 0);
  };
  auto R = [&](int i, hipStream_t s) { return nt ? rec_noted(e, i, s) : hipEventRecord(e[i], s); };
  if (which == 2) {  // ping-pong: b waits a, then a waits b
    CK(R(1, a));
    CK(W(b, e[1]));
    K(b, 1000);
    CK(R(2, b));
    CK(W(a, e[2]));
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
    CK(R(1, a));
    CK(W(b, e[1]));
    CK(R(2, b));
    CK(W(a, e[2]));  // a's own node reached through b
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
