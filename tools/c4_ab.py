"""C4 batches (n = 256, m = 64): A/B of a debug bit on the fused step (default
8192: the whole KKT assembled into K every step instead of the kept K0):
QP-steps/s at B = 1024 and 128, and the phase split.
    python tools/c4_ab.py [MASK]"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ipm-zoo_amd"))
import torch
import ipmz_amd as I

torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
ctx = I.Context(0)
for B in (1024, 128):
    MASK = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    for mask in (0, MASK, 0, MASK):
        I.debug_inject(mask)
        b = I.Batch(256, 64, 0, B, ctx)
        b.generate(1)
        flags = I.STEP_RESTART_IF_CONVERGED | I.STEP_GRAPH
        for _ in range(3):
            b.step(flags)
        ctx.sync()
        k = 20
        t0 = time.perf_counter()
        for _ in range(k):
            b.step(flags)
        ctx.sync()
        dt = (time.perf_counter() - t0) / k
        b.set_timing(True)
        for _ in range(5):
            b.step(I.STEP_RESTART_IF_CONVERGED)
        ph = b.phase_times()
        print(f"B {B} mask {mask}: {1e3 * dt:.3f} ms/step, {B / dt / 1e3:.1f} k QP-steps/s; phases (ms/step) " +
              " ".join(f"{kk} {ph[kk] / 5:.3f}" for kk in ("assemble", "factor", "solve", "eval")), flush=True)
        b.close()
I.debug_inject(0)
