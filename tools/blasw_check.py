"""C5 fp32 trailing update: SYRKX vs the halving tree (IPMZ_BLAS_W, read once
per process by the experiment build of profiles/r03_s5/blas_tree_ab.log; the
product has w = 512 built in, debug bit 1024 = SYRKX).  Prints the refinement statistics and the iterate after K steps
(saved to gpurun_out/blasw_<W>.npy for cross-run comparison), twice, and
whether the two runs are bitwise equal (determinism), then ms per step.
    IPMZ_BLAS_W=256 python tools/blasw_check.py"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ipm-zoo_amd"))
import numpy as np
import torch
import ipmz_amd as I

torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
ctx = I.Context(0)
W = os.environ.get("IPMZ_BLAS_W", "256")
n = int(os.environ.get("C5_N", 16384))
runs = []
for rep in range(2):
    qp = I.Optimizer(n, 0, 0, ctx)
    qp.generate(1234)
    qp.set_mixed_precision(True, 1e-12, 20)
    flags = I.STEP_RESTART_IF_CONVERGED
    for it in range(4):
        qp.step(flags)
        ctx.sync()
        s = qp.scalars()
        print(f"W={W} rep {rep} step {it}: ir aff {s['ir_iters_aff']:.0f} ratio {s['ir_ratio_aff']:.2e}, "
              f"corr {s['ir_iters']:.0f} ratio {s['ir_ratio']:.2e}", flush=True)
    runs.append(qp.vars())
    if rep == 0:
        k = 10
        t0 = time.perf_counter()
        for _ in range(k):
            qp.step(flags)
        ctx.sync()
        dt = (time.perf_counter() - t0) / k
        print(f"W={W}: {1e3 * dt:.3f} ms/step ({1 / dt:.2f} steps/s)", flush=True)
    qp.close()
print(f"W={W}: runs bitwise equal: {np.array_equal(runs[0], runs[1])}", flush=True)
os.makedirs("gpurun_out", exist_ok=True)
np.save(f"gpurun_out/blasw_{W}.npy", runs[1])
ref = "gpurun_out/blasw_0.npy"
if W != "0" and os.path.exists(ref):
    r = np.load(ref)
    print(f"W={W}: max |x - x_syrkx| / max |x_syrkx| = {np.max(np.abs(runs[1] - r)) / np.max(np.abs(r)):.3e}")
