"""A/B of a debug bit on whole Newton steps (production flags, eager or graph
as the step chooses): ms per step for C3 / C2 / C5 shapes.
    python tools/mask_ab.py MASK [workloads...]"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ipm-zoo_amd"))
import torch
import ipmz_amd as I

W = {"c3": (8192, 2048, 1024, {}), "c2": (2048, 512, 0, {"normal": 1}), "c5": (16384, 0, 0, {"mixed": 1})}
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
ctx = I.Context(0)
mask = int(sys.argv[1])
for wl in (sys.argv[2:] or ["c3", "c2", "c5"]):
    n, m, p, o = W[wl]
    for msk in (0, mask, 0, mask):
        I.debug_inject(msk)
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
        print(f"{wl} mask {msk}: {1e3 * dt:.3f} ms/step ({1 / dt:.2f} steps/s)", flush=True)
        qp.close()
I.debug_inject(0)
