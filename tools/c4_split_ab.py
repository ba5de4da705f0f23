"""C4 overlap probe: one Batch of 1024 QPs vs the same 1024 QPs as k Batches
of 1024/k on k contexts (streams), each step replaying k graphs that the
device may run side by side (one batch's memory-bound phases beside
another's factor).  ms per step of all 1024 QPs."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ipm-zoo_amd"))
import torch
import ipmz_amd as I

torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
n, m, p, B = 256, 64, 0, 1024
flags = I.STEP_RESTART_IF_CONVERGED | I.STEP_GRAPH
for k in (1, 2, 4, 1, 2, 4, 8):
    ctxs = [I.Context(0) for _ in range(k)]
    qps = [I.Batch(n, m, p, B // k, c) for c in ctxs]
    for i, q in enumerate(qps):
        q.generate(i * (B // k))
    for _ in range(3):
        for q in qps:
            q.step(flags)
    for c in ctxs:
        c.sync()
    steps = 20
    t0 = time.perf_counter()
    for _ in range(steps):
        for q in qps:
            q.step(flags)
    for c in ctxs:
        c.sync()
    dt = (time.perf_counter() - t0) / steps
    print(f"k={k}: {1e3 * dt:.3f} ms per step of {B} QPs ({B / dt / 1e3:.1f} k QP-steps/s), graph {qps[0].last_step_graph()}",
          flush=True)
    for q in qps:
        q.close()
    for c in ctxs:
        c.close()
