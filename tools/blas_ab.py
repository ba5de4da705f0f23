"""C5 (n = 16384, fp32 factor + fp64 refinement): rocBLAS SYRKX for the fp32
trailing update vs gemm_nt_kernel<float> (debug bit 128), ms per step and
the factor phase (instrumented pass).  Runs in the bench's process setup
(torch loaded first: its bundled rocBLAS is the one libipmz binds)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ipm-zoo_amd"))
import torch
import ipmz_amd as I

torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
ctx = I.Context(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
for mask in (0, 128, 0, 128):
    I.debug_inject(mask)
    qp = I.Optimizer(n, 0, 0, ctx)
    qp.generate(1234)
    qp.set_mixed_precision(True, 1e-12, 20)
    flags = I.STEP_RESTART_IF_CONVERGED | I.STEP_GRAPH
    for _ in range(2):
        qp.step(flags)
    ctx.sync()
    k = 8
    t0 = time.perf_counter()
    for _ in range(k):
        qp.step(flags)
    ctx.sync()
    dt = (time.perf_counter() - t0) / k
    qp.set_timing(True)
    for _ in range(3):
        qp.step(I.STEP_RESTART_IF_CONVERGED)
    ph = qp.phase_times()
    s = qp.scalars()
    print(f"mask {mask}: {1e3 * dt:.2f} ms/step ({1 / dt:.1f} steps/s), factor {ph['factor'] / 3:.2f} ms, "
          f"solve {ph['solve'] / 3:.2f} ms, ir {s['ir_iters_aff']:.0f}+{s['ir_iters']:.0f} ratio {s['ir_ratio']:.1e}",
          flush=True)
    qp.close()
I.debug_inject(0)
