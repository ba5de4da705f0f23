"""Repeated C5 (mixed-precision) and fp64 solves to convergence: a race in
the factor's hand-offs shows as a non-finite iterate or a failed solve."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "ipm-zoo_amd"))
import numpy as np
import torch
import ipmz_amd as I
torch.cuda.set_device(0)
ctx = I.Context(0)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for rep in range(reps):
    g = I.Optimizer(16384, 0, 0, ctx)
    g.generate(1234 + rep)
    g.set_mixed_precision(True, 1e-12, 20)
    iters, tr = g.solve(60)
    bad = [i for i, r in enumerate(tr) if not np.isfinite(r["f"])]
    print(f"C5 rep {rep}: iters {iters} converged {tr[-1]['converged']} first non-finite {bad[0] if bad else None}",
          flush=True)
    g.close()
    g = I.Optimizer(4096, 1024, 512, ctx)
    g.generate(7 + rep)
    iters, tr = g.solve(60)
    bad = [i for i, r in enumerate(tr) if not np.isfinite(r["f"])]
    print(f"  fp64 N=5632: iters {iters} converged {tr[-1]['converged']} first non-finite {bad[0] if bad else None}",
          flush=True)
    g.close()
print("mixed probe done", flush=True)
