#!/usr/bin/env python3
"""A/B: back-to-back eager steps vs a host sync after every step (queue depth).

    python tools/step_sync_ab.py [c2|c3] [steps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ipm-zoo_amd"))
import torch  # noqa: E402,F401  (one HIP runtime per process: torch first)
import ipmz_amd as I  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
n, m, p = {"c2": (2048, 512, 0), "c3": (8192, 2048, 1024)}[wl]
ctx = I.Context(0)
qp = I.Optimizer(n, m, p, ctx)
qp.generate(1234)
if wl == "c2":
    qp.set_reduction(I.REDUCTION_NORMAL)
flags = I.STEP_RESTART_IF_CONVERGED | I.STEP_GRAPH
for _ in range(3):
    qp.step(flags)
torch.cuda.synchronize()
for mode in ("async", "sync", "async", "sync"):
    t = time.perf_counter()
    for _ in range(steps):
        qp.step(flags)
        if mode == "sync":
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    print(f"{wl} {mode:5s} {1e3 * dt:8.3f} ms/step {1 / dt:8.1f} steps/s", flush=True)
