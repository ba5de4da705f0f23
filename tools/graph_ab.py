"""Eager (at most one step in flight) vs HIP-graph replay of whole Newton
steps whose factor forks onto the look-ahead streams (debug bit 4 lifts the
eager fallback): ms per step for C3, C2, C5 shapes.  Args: workloads."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ipm-zoo_amd"))
import torch
import ipmz_amd as I

W = {"c3": (8192, 2048, 1024, {}), "c2": (2048, 512, 0, {"normal": 1}), "c5": (16384, 0, 0, {"mixed": 1}),
     "s": (1024, 256, 128, {})}
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
ctx = I.Context(0)
for wl in (sys.argv[1:] or ["c2", "c3", "c5"]):
    n, m, p, o = W[wl]
    for mode in ("eager", "graph", "eager", "graph"):
        I.debug_inject(I.INJECT_GRAPH_FORKS if mode == "graph" else 0)
        qp = I.Optimizer(n, m, p, ctx)
        qp.generate(1234)
        if o.get("mixed"):
            qp.set_mixed_precision(True, 1e-12, 20)
        if o.get("normal"):
            qp.set_reduction(I.REDUCTION_NORMAL)
        flags = I.STEP_RESTART_IF_CONVERGED | I.STEP_GRAPH
        for _ in range(2):
            qp.step(flags)
        ctx.sync()
        k = 10
        t0 = time.perf_counter()
        for _ in range(k):
            qp.step(flags)
        ctx.sync()
        dt = (time.perf_counter() - t0) / k
        print(f"{wl} {mode}: {1e3 * dt:.3f} ms/step (graph replayed: {qp.last_step_graph()})", flush=True)
        qp.close()
I.debug_inject(0)
