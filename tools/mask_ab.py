"""A/B of a debug bit on whole Newton steps (production flags, eager or graph
as the step chooses): ms per step for C3 / C2 / C5 shapes.
    [TORCH_STREAM=1] python tools/mask_ab.py MASK [workloads...]"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("IPMZ_PKG_DIR") or os.path.join(REPO, "ipm-zoo_amd"))  # IPMZ_PKG_DIR: another build
import torch
import ipmz_amd as I

W = {"c3": (8192, 2048, 1024, {}), "c2": (2048, 512, 0, {"normal": 1}), "c5": (16384, 0, 0, {"mixed": 1})}
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
# TORCH_STREAM=1: on torch's current (default) stream, as bench.py; 2: on a torch side stream
TS = os.environ.get("TORCH_STREAM", "0")
side = torch.cuda.Stream() if TS == "2" else None
if side is not None:
    torch.cuda.set_stream(side)
ctx = I.Context(0, stream=torch.cuda.current_stream().cuda_stream) if TS in ("1", "2") else I.Context(0)
print("ctx stream", torch.cuda.current_stream().cuda_stream if TS != "0" else "own", flush=True)
if os.environ.get("AB_NBO"):  # AB_NBO=384: that outer panel width (else by matrix order)
    ctx.set_blocking(int(os.environ["AB_NBO"]), 64)
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
        # STEP_STREAM=own|torch: step on another stream than the one the QP was made on
        if os.environ.get("STEP_STREAM") == "own":
            ctx.sync()
            ctx.set_stream(None)
        elif os.environ.get("STEP_STREAM") == "torch":
            ctx.sync()
            ctx.set_stream(torch.cuda.current_stream().cuda_stream)
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
        if os.environ.get("STEP_STREAM"):
            ctx.set_stream(torch.cuda.current_stream().cuda_stream if TS in ("1", "2") else None)
I.debug_inject(0)
